// EXPERIMENT (not in the product build): register-resident pass 3 for
// L3 = 256, measured slower than the LDS-staged pass3_kernel of
// csrc/hip/fft_passes.hip -- numbers in profiles/pass3r_register_r2.txt.
// To try it again, paste the kernel and launcher below into fft_passes.hip
// (after pass3_kernel; it uses P3Emit, row_base, row_twiddles from there) and
// put the dispatch block at the top of launch_pass3.

// Register-resident pass 3 for L3 = 256 = 16 x 16. One 16-lane group owns one
// row: lane t loads elements t + 16 q (128-B row pieces), does the stage-1
// DFT16 and its twiddle W_256^{t k1} in registers, and exchanges with the
// other 15 lanes of its group through a wave-private LDS block (one write +
// one read per element, no workgroup barrier); stage 2 leaves bins
// k3 = t + 16 k2 of the row in lane t. A wave holds two row pairs
// (c, C - c) in lanes 0-15 / 16-31 and 32-47 / 48-63: the untangle partner of
// bin k3, bin 255 - k3 of the mirror row, sits in lane ^ 31, register
// 15 - k2, and comes over with one ds_bpermute per word. Rows 0 and C/2 are
// their own mirrors and share one pair slot (pair 0): row C/2 takes lane
// 15 - t, row 0 lane (16 - t) mod 16 (lane 0 of row 0 rotates its own
// registers). The power spectrum goes through an LDS image so that the
// stores are runs of PAIRS consecutive rows. Against pass3_kernel (LDS-staged
// DFT stages): 3 instead of 8 LDS accesses per bin, fewer registers.
template <int PAIRS, int MODE, int WPE>
__global__ void __launch_bounds__(PAIRS * 32) __attribute__((amdgpu_waves_per_eu(WPE, 8))) pass3r_kernel(Pass3Args a) {
  constexpr int L = 256;
  constexpr int L4 = 4 * L;
  constexpr int kT4 = 32 + L4 / 32;
  constexpr int NT = PAIRS * 32;
  constexpr int kGrp = 16 * 17;  // floats per group: pitch 17 (odd -> conflict-free column writes), == 16 mod 32
  constexpr int kSp = PAIRS + 1;          // staging image pitch (floats)
  constexpr int kSide = L * kSp + 16;     // staging side stride (== 16 mod 32: the two sides of a pair on distinct banks)
  constexpr int kXch = (2 * PAIRS * kGrp > 2 * kSide ? 2 * PAIRS * kGrp : 2 * kSide) / 2;  // float2
  constexpr bool kPower = (MODE == P3_POWER || MODE == P3_POWER16);
  __shared__ __attribute__((aligned(16))) float2 xch[kXch];
  __shared__ float2 twl[kTwPad<L>];
  __shared__ float2 t4[kT4];
  auto w4 = [&](uint32_t j) { return cmul(t4[32 + (j >> 5)], t4[j & 31u]); };

  const int b = blockIdx.y;
  const int lane = threadIdx.x & 63;
  const int t = lane & 15;
  const int side = (lane >> 4) & 1;       // 0: row c, 1: its mirror
  const int grp = threadIdx.x >> 4;       // group of the workgroup
  const int pl = threadIdx.x >> 5;        // pair of the workgroup
  const uint32_t half = a.C / 2;
  const uint32_t pair = xcd_remap(blockIdx.x, gridDim.x) * PAIRS + pl;
  const bool valid = pair < half;
  const bool special = pair == 0;         // rows 0 and C/2
  const uint32_t pc = valid ? pair : 1u;
  const uint32_t row = special ? (side ? half : 0u) : (side ? a.C - pc : pc);

  const float2* src = a.buf + static_cast<size_t>(b) * a.M + row_base(row, a.L1, a.L2, a.L3) + t;
  float2 z[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) z[q] = src[16 * q];
  copy_stage_twiddles<L>(twl, a.tb.st3);
  for (int i = threadIdx.x; i < kT4; i += NT) t4[i] = a.tb.p3[i];
  double delta = 0.0;
  uint32_t n_s = 0;
  if (kPower) {
    n_s = a.tmpl[b].n_steps;
    delta = a.delta[b];
  }
  const RowTw rt = row_twiddles(a.tw, row, n_s);
  __syncthreads();

  // stage 1: DFT16 over q of x[t + 16 q], then W_256^{t k1}
  Dft<16>::run(z);
#pragma unroll
  for (int k1 = 1; k1 < 16; ++k1) {
    const int e = (t * k1) & (L - 1);
    z[k1] = cmul(z[k1], twl[e + (e >> 4)]);
  }
  // exchange inside the group: lane t writes (t, k1), reads column k1 = t.
  // LDS operations of one wave complete in order; the fences only keep the
  // compiler from moving them.
  // Real and imaginary parts cross separately (half the LDS per wave: the
  // block, not the VGPRs, would otherwise cap the occupancy at 4 waves/SIMD).
  float* xg = reinterpret_cast<float*>(xch) + grp * kGrp;
  auto wave_sync = [] {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_wave_barrier();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
  };
#pragma unroll
  for (int k1 = 0; k1 < 16; ++k1) xg[t * 17 + k1] = z[k1].x;
  wave_sync();
#pragma unroll
  for (int j = 0; j < 16; ++j) z[j].x = xg[j * 17 + t];
  wave_sync();
#pragma unroll
  for (int k1 = 0; k1 < 16; ++k1) xg[t * 17 + k1] = z[k1].y;
  wave_sync();
#pragma unroll
  for (int j = 0; j < 16; ++j) z[j].y = xg[j * 17 + t];
  // stage 2: DFT16 over j -> z[k2] = Z_row[t + 16 k2]
  Dft<16>::run(z);

  // untangle partner of bin k3 = t + 16 k2: bin 255 - k3 of the mirror row
  // (lane ^ 31, register 15 - k2); row C/2: lane 15 - t of its own group;
  // row 0: lane (16 - t) mod 16, and for t == 0 register (16 - k2) mod 16 of
  // the lane itself
  const int gbase = lane & ~15;
  const int plane = special ? gbase + (side ? 15 - t : ((16 - t) & 15)) : (lane ^ 31);
  const bool rot = special && side == 0 && t == 0;
  auto partner = [&](int k2) -> float2 {
    const float2 v = z[15 - k2];
    float2 r;
    r.x = __int_as_float(__builtin_amdgcn_ds_bpermute(plane << 2, __float_as_int(v.x)));
    r.y = __int_as_float(__builtin_amdgcn_ds_bpermute(plane << 2, __float_as_int(v.y)));
    return rot ? z[(16 - k2) & 15] : r;
  };

  const bool correct = kPower && n_s > 0;
  P3Emit<MODE> emit{a, static_cast<float>(delta), correct, b};
  // W_2N^k for k = row + C k3, k3 = t + 16 k2: exact at k2 = 0 and k2 = 8,
  // stepped by W_{4L}^16 in between (at most 7 rotations)
  const float2 tk_step = w4(16u);
  float2 tk_lo = cmul(rt.t1, w4(static_cast<uint32_t>(t)));
  float2 tk_hi = cmul(rt.t1, w4(static_cast<uint32_t>(t + 128)));
  float2 ta_lo = make_float2(0.f, 0.f), ta_hi = ta_lo, ta_step = make_float2(1.f, 0.f);
  if (correct) {
    ta_lo = cmul(rt.ta, w4((n_s * static_cast<uint32_t>(t)) % L4));
    ta_hi = cmul(rt.ta, w4((n_s * static_cast<uint32_t>(t + 128)) % L4));
    ta_step = w4((n_s * 16u) % L4);
  }
  // power image [side][k3][pair] (reuses the exchange blocks: barrier first)
  float* stage = reinterpret_cast<float*>(xch);
  if constexpr (kPower) __syncthreads();
  auto bin = [&](int k2, float2 tk, float2 ta) {
    const int k3 = t + 16 * k2;
    const float2 zm = partner(k2);
    const uint32_t k = row + a.C * static_cast<uint32_t>(k3);
    const float2 x = untangle_w(z[k2], zm, cmul(tk, tk));  // W_N^k = tk^2
    if constexpr (kPower) {
      stage[side * kSide + k3 * kSp + pl] = emit.power(k, x, tk, ta);
    } else {
      if (valid) emit(k, x, tk, ta);
    }
  };
#pragma unroll
  for (int k2 = 0; k2 < 8; ++k2) {
    if (k2 > 0) {
      tk_lo = cmul(tk_lo, tk_step);
      tk_hi = cmul(tk_hi, tk_step);
      if (correct) {
        ta_lo = cmul(ta_lo, ta_step);
        ta_hi = cmul(ta_hi, ta_step);
      }
    }
    bin(k2, tk_lo, ta_lo);
    bin(k2 + 8, tk_hi, ta_hi);
  }
  if (valid && special && side == 0 && t == 0) emit.nyquist(z[0], n_s);
  if constexpr (kPower) {
    __syncthreads();
    const int cl = threadIdx.x % PAIRS;
    const uint32_t pp = pair - pl + cl;
    const bool ok = pp < half;
    const uint32_t rowa = pp, rowb = pp == 0 ? half : a.C - pp;
#pragma unroll 4
    for (int seg = threadIdx.x / PAIRS; seg < 2 * L; seg += NT / PAIRS) {
      const int sd = seg / L;
      const int k3 = seg % L;
      const float p = stage[sd * kSide + k3 * kSp + cl];
      const uint32_t k = (sd ? rowb : rowa) + a.C * static_cast<uint32_t>(k3);
      if (ok && k < a.limit) emit.store(k, p);
    }
  }
}


template <int PAIRS, int WPE>
hipError_t launch_pass3r(Pass3Mode mode, const Pass3Args& a, int batch, hipStream_t s) {
  const dim3 grid((a.C / 2 + PAIRS - 1) / PAIRS, batch);
  const dim3 block(PAIRS * 32);
  if (mode == P3_POWER && a.ps16) hipLaunchKernelGGL((pass3r_kernel<PAIRS, P3_POWER16, WPE>), grid, block, 0, s, a);
  else if (mode == P3_POWER) hipLaunchKernelGGL((pass3r_kernel<PAIRS, P3_POWER, WPE>), grid, block, 0, s, a);
  else hipLaunchKernelGGL((pass3r_kernel<PAIRS, P3_COMPLEX, WPE>), grid, block, 0, s, a);
  return hipGetLastError();
}


// dispatch (top of launch_pass3):
#if 0
  if (plan.L3 == 256 && a.L3 == 256 && a.C == plan.L1 * plan.L2 && a.C % 2 == 0) {
    // p3_pairs: row pairs per workgroup (4, 8); +100: at least 5 waves/SIMD (96 VGPRs)
    switch (plan.p3_pairs) {
      case 4: return launch_pass3r<4, 1>(mode, a, batch, s);
      case 8: return launch_pass3r<8, 1>(mode, a, batch, s);
      case 104: return launch_pass3r<4, 5>(mode, a, batch, s);
      case 108: return launch_pass3r<8, 5>(mode, a, batch, s);
      default: break;
    }
  }
#endif
