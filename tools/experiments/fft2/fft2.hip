// Two-pass template FFT (index algebra: fft2_kernels.hpp). Replaces, for the
// production shape, the reference's cuFFT / clFFT / FFTW template transform and
// its resampling + power-spectrum kernels (cuda/app/demod_binary_cuda.cu:849-965,
// opencl/app/demod_binary_ocl.cpp:972-1314, demod_binary_fft_fftw.c:46-113,
// cuda/app/demod_binary_cuda.cuh:69-184).
//
// Sized for CDNA4 occupancy rather than for one LDS-resident tile per pass:
//   pass A: a 768-point column with rows >= 256 in the padding is three
//           256-point DFTs of pre-twiddled data (X[s + 3k'] = DFT256(x W_768^{ns})),
//           so a 16-thread column group gathers its 16 samples once and runs the
//           three DFTs through one 35 KB LDS exchange buffer;
//   pass B: the two rows of a pair go through the same 70 KB row buffer one
//           after the other (two workgroups per CU, the whole grid resident);
//           the last stage of the mirror row is assigned reversed (butterfly
//           511 - t), so every thread ends with both partners of its untangle
//           pairs in registers and no final exchange is needed.
#include <algorithm>

#include "fft2_kernels.hpp"
#include "fft_block.hpp"

namespace brp {
namespace hipk {

namespace {

constexpr int kL1 = static_cast<int>(kFft2L1);
constexpr int kR = static_cast<int>(kFft2R);
constexpr int kCA = static_cast<int>(kFft2ColsA);
constexpr int kThrA = kCA * 16;
constexpr int kThrB = 512;
static_assert(kFft2PartialsA == kThrB, "pass B reduces one pass-A partial per thread");

// ------------------------------------------------------------------ pass A
// LDS element (e, c) of the 256-point exchange: the 4 j-groups of a wave land
// on alternating bank halves for both the stride-16 writes and stride-1 reads.
__device__ __forceinline__ int a_idx(int e, int c) { return kCA * e + c + kCA * (e >> 4); }
constexpr int kLdsA = kCA * 256 + kCA * 16;

// Thread (c = tid % 16, j = tid / 16): column n' = 16 blockIdx.x + c.
//   gather  rows n1 = j + 16 q (q < 16) of the column (the data third);
//   for s < 3: stage 1 (radix 16, Ns 1) of x[n1] W_768^{n1 s} in registers,
//           exchange, stage 2 (radix 16, Ns 16, twiddle W_256^{j q}): outputs
//           k' = j + 16 q, i.e. rows k1 = s + 3 j + 48 q, stored with W_M^{n' k1}.
__global__ void __launch_bounds__(kThrA) __attribute__((amdgpu_waves_per_eu(4))) colA_kernel(ColAArgs a) {
  __shared__ __attribute__((aligned(16))) float2 data[kLdsA];
  __shared__ float2 w768[kL1];
  __shared__ float lut_s[kLutSize], lut_c[kLutSize];
  __shared__ double red[kThrA / kWave + 1];

  const int b = blockIdx.y;
  const int c = threadIdx.x % kCA;
  const int j = threadIdx.x / kCA;
  const uint32_t ncol = blockIdx.x * kCA + c;
  if (a.reset != nullptr && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) *a.reset = 0;
  for (int i = threadIdx.x; i < kLutSize; i += kThrA) {
    lut_s[i] = kSinLut[i];
    lut_c[i] = kCosLut[i];
  }
  for (int e = threadIdx.x; e < kL1; e += kThrA) w768[e] = a.w768[e];
  __syncthreads();

  // nearest-neighbour resampling with the reference's float arithmetic; three
  // phases (indices, loads, centring) keep all 32 loads of the thread in flight
  const bool fast = a.n_unpadded <= (1u << 23);
  const TemplateDev td = a.tmpl[b];
  const float* series = a.series + static_cast<size_t>(td.wu) * a.n_unpadded;
  const int last = static_cast<int>(a.n_unpadded) - 1;
  int idx[32];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const uint32_t m0 = 2u * (static_cast<uint32_t>(j + 16 * q) * kR + ncol);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint32_t m = m0 + h;
      int i = -1;
      if (m < td.n_steps) {
        const float dt = resamp_del_t(m, td.p, lut_s, lut_c);
        i = min(max(fast ? resamp_nearest_f(m, dt) : resamp_nearest(m, dt), 0), last);
      }
      idx[2 * q + h] = i;
    }
  }
  float raw[32];
#pragma unroll
  for (int e = 0; e < 32; ++e) raw[e] = series[idx[e] < 0 ? 0 : idx[e]];
  float fsum = 0.0f;
  float2 x[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const float x0 = idx[2 * q] < 0 ? 0.0f : raw[2 * q] - td.mu0;
    const float x1 = idx[2 * q + 1] < 0 ? 0.0f : raw[2 * q + 1] - td.mu0;
    fsum += x0 + x1;
    x[q] = make_float2(x0, x1);
  }

  float2* out = a.out + static_cast<size_t>(b) * kFft2M + ncol;
  const float2 step = tw_lookup32(a.tw, 4u * 48u * ncol);  // W_M^{48 n'}
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    float2 y[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) y[q] = (s == 0) ? x[q] : cmul(x[q], w768[(s * (j + 16 * q)) % kL1]);
    Dft<16>::run(y);
    if (s > 0) __syncthreads();  // previous s has read the exchange buffer
#pragma unroll
    for (int q = 0; q < 16; ++q) data[a_idx(16 * j + q, c)] = y[q];
    __syncthreads();
    float2 z[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) z[q] = data[a_idx(j + 16 * q, c)];
#pragma unroll
    for (int q = 1; q < 16; ++q) z[q] = cmul(z[q], w768[3 * j * q]);  // W_256^{j q}
    Dft<16>::run(z);
    // rows k1 = k0 + 48 q; W_M^{n' k1} exact at q = 0 and 8, stepped in between
    const uint32_t k0 = static_cast<uint32_t>(s + 3 * j);
    float2 t0 = tw_lookup32(a.tw, 4u * ncol * k0);
    float2 t8 = tw_lookup32(a.tw, 4u * ncol * (k0 + 384u));
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      out[static_cast<size_t>(k0 + 48u * q) * kR] = cmul(z[q], t0);
      out[static_cast<size_t>(k0 + 48u * (q + 8)) * kR] = cmul(z[q + 8], t8);
      t0 = cmul(t0, step);
      t8 = cmul(t8, step);
    }
  }
  const double tot = block_sum<kThrA>(static_cast<double>(fsum), red);
  if (threadIdx.x == 0) a.partials[static_cast<size_t>(b) * gridDim.x + blockIdx.x] = tot;
}

// ------------------------------------------------------------------ pass B
// Row buffer index: two pad elements every 32 keep the float4 stage-1 writes,
// the contiguous stage reads and the stride-2 / stride-32 Stockham scatters at
// the 2 (b64) or 4 (b128) LDS cycles per wave instruction minimum.
__device__ __forceinline__ int b_idx(int e) { return e + 2 * (e >> 5); }
constexpr int kLdsB = kR + 2 * (kR >> 5);

// One 8192-point row, radices 2, 16, 16, 16 (Stockham, natural order). On
// entry v[2u], v[2u+1] = row[t + 512 u], row[t + 512 u + 4096]; on exit
// v[q] = X[jl + 512 q] (jl = this thread's last-stage butterfly).
__device__ __forceinline__ void rowB_fft(float2 (&v)[16], int jl, float2* data, const float2* w512,
                                         const float2* w8k) {
  // an opaque copy of the thread index: without it the compiler shares the
  // LDS address arithmetic of the two inlined row transforms and keeps ~60
  // VGPRs of addresses live (spilled) from the first row to the second
  int t = threadIdx.x;
  asm volatile("" : "+v"(t), "+v"(jl));
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const float2 p = v[2 * u], q = v[2 * u + 1];
    v[2 * u] = cadd(p, q);
    v[2 * u + 1] = csub(p, q);
  }
  __syncthreads();  // the row buffer is free
#pragma unroll
  for (int u = 0; u < 8; ++u)
    *reinterpret_cast<float4*>(&data[b_idx(2 * (t + 512 * u))]) =
        make_float4(v[2 * u].x, v[2 * u].y, v[2 * u + 1].x, v[2 * u + 1].y);
  __syncthreads();
  // radix 16, Ns 2: twiddle W_32^{(t % 2) q} = W_512^{16 (t % 2) q}
#pragma unroll
  for (int q = 0; q < 16; ++q) v[q] = data[b_idx(t + 512 * q)];
  if (t & 1) {
#pragma unroll
    for (int q = 1; q < 16; ++q) v[q] = cmul(v[q], w512[16 * q]);
  }
  Dft<16>::run(v);
  __syncthreads();
  {
    const int base = (t >> 1) * 32 + (t & 1);
#pragma unroll
    for (int q = 0; q < 16; ++q) data[b_idx(base + 2 * q)] = v[q];
  }
  __syncthreads();
  // radix 16, Ns 32: twiddle W_512^{(t % 32) q}
#pragma unroll
  for (int q = 0; q < 16; ++q) v[q] = data[b_idx(t + 512 * q)];
#pragma unroll
  for (int q = 1; q < 16; ++q) v[q] = cmul(v[q], w512[(t & 31) * q]);
  Dft<16>::run(v);
  __syncthreads();
  {
    // The last stage's twiddle W_8192^{jl q} of element e = jl + 512 q depends
    // on e only, so it is applied here by the writer: e = base + 32 q' has
    // jl = t % 32 + 32 q', q = t / 32 = g, W_8192^{jl g} = W_8192^{(t%32) g} W_256^{g q'}.
    // (The reader would hold 15 twiddles at once; the writer streams them.)
    const int base = (t >> 5) * 512 + (t & 31);
    const int g = t >> 5;
    const float2 c = w8k[(t & 31) * g];
#pragma unroll
    for (int q = 0; q < 16; ++q) data[b_idx(base + 32 * q)] = cmul(v[q], q == 0 ? c : cmul(c, w512[2 * g * q]));
  }
  __syncthreads();
  // radix 16, Ns 512: butterfly jl (twiddles applied by the writer)
#pragma unroll
  for (int q = 0; q < 16; ++q) v[q] = data[b_idx(jl + 512 * q)];
  Dft<16>::run(v);
}

// One workgroup per row pair (k1, 768 - k1), k1 = 0 .. 384 (rows 0 and 384
// pair with themselves). Thread t owns bins m = t + 512 q of row k1 and,
// through the reversed last stage, their untangle partners in the mirror row:
// R - 1 - m in general, (R - m) mod R for row 0.
__global__ void __launch_bounds__(kThrB) __attribute__((amdgpu_waves_per_eu(4))) rowB_kernel(RowBArgs a) {
  __shared__ __attribute__((aligned(16))) float2 data[kLdsB];
  __shared__ float2 w512[512];
  __shared__ double red[kThrB / kWave + 1];

  const int b = blockIdx.y;
  const uint32_t k1 = blockIdx.x;
  const uint32_t k1m = (kFft2L1 - k1) % kFft2L1;
  const bool row0 = (k1 == 0);
  const bool self = row0 || k1 == kFft2L1 / 2;
  const int t = threadIdx.x;
  const int pb = row0 ? ((512 - t) & 511) : 511 - t;
  float2* base = a.buf + static_cast<size_t>(b) * kFft2M;
  // row loads: stage 1 reads elements t + 512 u and t + 512 u + 4096
  auto load_row = [&](float2 (&v)[16], uint32_t row) {
    const float2* r = base + static_cast<size_t>(row) * kR;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      v[2 * u] = r[t + 512 * u];
      v[2 * u + 1] = r[t + 512 * u + 4096];
    }
  };
  float2 va[16], vb[16];
  load_row(va, k1);
  w512[t] = a.w512[t];
  // mean-padding correction delta = (sum of (sample - mu0)) / n_steps, the
  // same fixed-order reduction in every workgroup
  const uint32_t n_s = a.tmpl[b].n_steps;
  const double tot = block_sum<kThrB>(a.partials[static_cast<size_t>(b) * kFft2PartialsA + t], red);
  const float dS = n_s ? static_cast<float>(tot / static_cast<double>(n_s)) : 0.0f;

  // the mirror row is loaded after the first row's transform (the second
  // resident workgroup of the CU covers the latency): 128 VGPRs, 4 waves/SIMD
  rowB_fft(va, t, data, w512, a.w8k);
  // park the first row's transform in its own (consumed) storage while the
  // mirror row is transformed: holding both in registers would exceed the
  // 128-VGPR budget of two resident workgroups per CU and spill to scratch
  // mirror row first: for rows 0 and 384 it is this row's own storage. The
  // thread parks to exactly the elements it loaded (t + 512 q), and waits for
  // its loads before overwriting them.
  float2* park = base + static_cast<size_t>(k1) * kR;
  load_row(vb, k1m);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int q = 0; q < 16; ++q) park[t + 512 * q] = va[q];
  rowB_fft(vb, pb, data, w512, a.w8k);
#pragma unroll
  for (int q = 0; q < 16; ++q) va[q] = park[t + 512 * q];

  // untangle + power. Both rows' complex data were consumed into registers
  // above, so the spectrum goes to the first half of their own storage.
  const bool correct = n_s > 0;
  float* psa = reinterpret_cast<float*>(base + static_cast<size_t>(k1) * kR);
  float* psb = reinterpret_cast<float*>(base + static_cast<size_t>(k1m) * kR);
  auto power = [&](uint32_t k, float2 x, float2 tk, float2 ta) -> float {
    if (k == 0) return 0.0f;
    if (correct) {
      const float ratio = ta.y * __builtin_amdgcn_rcpf(tk.y);  // v_rcp_f32 (1 ulp)
      const float2 tc = cmul(ta, conjf2(tk));                  // W_2N^{(n_s-1) k}
      x = make_float2(x.x - dS * ratio * tc.x, x.y - dS * ratio * tc.y);
    }
    return (x.x * x.x + x.y * x.y) * a.norm;
  };
  // W_2N^k and W_2N^{n_s k} of k = k1 + 768 m, m = t + 512 q: exact at q = 0
  // and 8, stepped by W_2N^{768 * 512} (n_s times) in between
  // (period 2N = 4M is a compile-time constant here: the reductions compile to
  // multiply-shift sequences)
  constexpr uint64_t kP = 4ull * kFft2M;
  constexpr uint32_t kStep = kFft2L1 * 512u;
  const uint32_t ka = k1 + kFft2L1 * static_cast<uint32_t>(t);
  const uint32_t kb = ka + kFft2L1 * 4096u;
  float2 tkA = tw_lookup32(a.tw, ka), tkB = tw_lookup32(a.tw, kb);
  const float2 tk_step = tw_lookup32(a.tw, kStep);
  float2 taA = make_float2(1.f, 0.f), taB = taA, ta_step = taA;
  if (correct) {
    taA = tw_lookup32(a.tw, static_cast<uint32_t>(static_cast<uint64_t>(n_s) * ka % kP));
    taB = tw_lookup32(a.tw, static_cast<uint32_t>(static_cast<uint64_t>(n_s) * kb % kP));
    ta_step = tw_lookup32(a.tw, static_cast<uint32_t>(static_cast<uint64_t>(n_s) * kStep % kP));
  }
  const bool zero_lane = row0 && t == 0;  // m = 512 q pairs with 512 ((16 - q) mod 16)
  auto bin = [&](int q, float2 zm, float2 tk, float2 ta) {
    const uint32_t m = static_cast<uint32_t>(t) + 512u * q;
    const uint32_t k = k1 + kFft2L1 * m;
    const float2 zk = va[q];
    const float2 w = cmul(tk, tk);  // W_N^k
    if (k < a.limit) psa[m] = power(k, untangle_w(zk, zm, w), tk, ta);
    if (!self) {
      // bin M - k = k1m + 768 (R - 1 - m): W_N^{M-k} = -conj(W_N^k),
      // W_2N^{M-k} = -i conj(W_2N^k), W_2N^{n_s (M-k)} = (-i)^{n_s} conj(W_2N^{n_s k})
      const uint32_t mm = kR - 1 - m;
      const uint32_t kk = k1m + kFft2L1 * mm;
      if (kk < a.limit)
        psb[mm] = power(kk, untangle_w(zm, zk, make_float2(-w.x, w.y)), make_float2(-tk.y, -tk.x),
                        rot_mi(conjf2(ta), n_s));
    }
  };
#pragma unroll
  for (int h = 0; h < 8; ++h) {
    if (h > 0) {
      tkA = cmul(tkA, tk_step);
      tkB = cmul(tkB, tk_step);
      if (correct) {
        taA = cmul(taA, ta_step);
        taB = cmul(taB, ta_step);
      }
    }
    // select values, not array elements (keeps vb in registers)
    const float2 z0a = vb[(16 - h) & 15], z0b = vb[15 - h];
    const float2 z8a = vb[(8 - h) & 15], z8b = vb[7 - h];
    bin(h, zero_lane ? z0a : z0b, tkA, taA);
    bin(h + 8, zero_lane ? z8a : z8b, tkB, taB);
  }
  if (zero_lane && kFft2M < a.limit) {
    // Nyquist bin M: X_M = Re Z_0 - Im Z_0 (natural order)
    float2 x = make_float2(va[0].x - va[0].y, 0.0f);
    if (correct) {
      const float2 sp = padding_spectrum_t(
          tw_lookup32(a.tw, static_cast<uint32_t>(static_cast<uint64_t>(n_s) * kFft2M % kP)), tw_lookup32(a.tw, kFft2M),
          tw_lookup32(a.tw, static_cast<uint32_t>(static_cast<uint64_t>(n_s - 1) * kFft2M % kP)));
      x = make_float2(x.x + dS * sp.x, x.y + dS * sp.y);
    }
    const float pm = (x.x * x.x + x.y * x.y) * a.norm;
    if (a.ps16) a.ps16[static_cast<size_t>(b) * a.ps_stride + kFft2M] = static_cast<_Float16>(pm);
    else a.ps[static_cast<size_t>(b) * a.ps_stride + kFft2M] = pm;
  }
}

// ------------------------------------------------------------------ pass T
// PS[k] = slab[k % 768][k / 768] for k < min(limit, M); 64 x 64 tiles via LDS.
template <bool HALF>
__global__ void __launch_bounds__(256) psT_kernel(PsTArgs a) {
  __shared__ float tile[64][65];
  const int b = blockIdx.z;
  const uint32_t r0 = blockIdx.x * 64;  // k1
  const uint32_t m0 = blockIdx.y * 64;  // m
  const float* src = reinterpret_cast<const float*>(a.buf + static_cast<size_t>(b) * kFft2M);
  const int tx = threadIdx.x % 16, ty = threadIdx.x / 16;
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int r = ty + 16 * rr;
    const float4 v = *reinterpret_cast<const float4*>(src + static_cast<size_t>(r0 + r) * (2 * kR) + m0 + 4 * tx);
    tile[r][4 * tx + 0] = v.x;
    tile[r][4 * tx + 1] = v.y;
    tile[r][4 * tx + 2] = v.z;
    tile[r][4 * tx + 3] = v.w;
  }
  __syncthreads();
  const uint32_t kmax = a.limit < kFft2M ? a.limit : kFft2M;
  const int lane = threadIdx.x % 64, w = threadIdx.x / 64;
#pragma unroll
  for (int mm = 0; mm < 16; ++mm) {
    const int m = w + 4 * mm;
    const uint32_t k = r0 + lane + kFft2L1 * (m0 + m);
    if (k < kmax) {
      const float v = tile[lane][m];
      if (HALF) a.ps16[static_cast<size_t>(b) * a.ps_stride + k] = static_cast<_Float16>(v);
      else a.ps[static_cast<size_t>(b) * a.ps_stride + k] = v;
    }
  }
}

}  // namespace

hipError_t launch_colA(const ColAArgs& a, int batch, hipStream_t s) {
  hipLaunchKernelGGL(colA_kernel, dim3(kR / kCA, batch), dim3(kThrA), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_rowB(const RowBArgs& a, int batch, hipStream_t s) {
  hipLaunchKernelGGL(rowB_kernel, dim3(kFft2L1 / 2 + 1, batch), dim3(kThrB), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_psT(const PsTArgs& a, int batch, hipStream_t s) {
  const uint32_t kmax = std::min(a.limit, kFft2M);
  const uint32_t mrows = (kmax + kFft2L1 - 1) / kFft2L1;  // m < mrows hold bins < kmax
  if (mrows == 0) return hipSuccess;
  const dim3 grid(kFft2L1 / 64, (mrows + 63) / 64, batch);
  if (a.ps16) hipLaunchKernelGGL(psT_kernel<true>, grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL(psT_kernel<false>, grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace hipk
}  // namespace brp
