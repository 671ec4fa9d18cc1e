// Two-pass template FFT for the production shape (N = 3 * 2^22 after 3x
// padding, M = N/2 = 768 * 8192 complex points) plus a power-spectrum
// transpose. Compared with the three-pass transform (fft_passes.hip) the
// 50 MB complex intermediate crosses HBM once instead of twice:
//
//   pass A (colA_kernel): resampling gather fused into 768-point column FFTs
//     over n1 (stride R = 8192), output row k1 of length R written contiguous,
//     twiddled by W_M^{n' k1};
//   pass B (rowB_kernel): one workgroup per row pair (k1, 768 - k1): 8192-point
//     row FFTs in LDS (radix 16, 16, 16, 2), the real-FFT untangle of the two
//     rows, the analytic mean-padding correction and |X|^2 / N, written in
//     slab-major order PSs[k1][m] for bin k = k1 + 768 m (contiguous stores);
//   transpose (psT_kernel): PSs -> natural bin order for the harmonic sum
//     (21 MB, Infinity-Cache resident between pass B and the harmonic sum).
//
// Index algebra: n = n1 R + n', k = k1 + L1 m (L1 = 768, R = 8192):
//   X[k1 + L1 m] = sum_n' W_R^{n' m} W_M^{n' k1} sum_n1 z[n1 R + n'] W_L1^{n1 k1}.
// Pass A needs padding >= 3 (rows n1 >= 256 are zero: stage 1 replicates, as
// in pass1_pruned3_kernel). Replaces the reference's cuFFT/clFFT/FFTW calls and
// resampling kernels (cuda/app/demod_binary_cuda.cu:416-965,
// opencl/app/demod_binary_ocl.cpp:487-1314, demod_binary_fft_fftw.c:88-113).
#include <algorithm>

#include "fft2_kernels.hpp"
#include "fft_block.hpp"

namespace brp {
namespace hipk {

namespace {

constexpr int kL1 = kFft2L1;  // 768 = 3 * 16 * 16
constexpr int kR = kFft2R;    // 8192 = 16 * 16 * 16 * 2
constexpr int kCols = 16;     // pass A columns per workgroup (128-B row segments)
constexpr int kThrA = kCols * 48;  // 48 threads per column: one radix-16 butterfly each
constexpr int kThrB = 1024;        // 512 threads per row of the pair

// ------------------------------------------------------------------ pass A
// Thread (c = tid % 16, j = tid / 16 < 48).
//   gather:   rows r = j + 48 u < 256 of column c (the data third; rows >= 256
//             are zero padding), LUT-sine nearest-neighbour resampling;
//   stage 2:  radix-16 butterfly j (Ns = 3) after the replicating radix-3
//             stage: inputs x[g + 16 q], g = j / 3, twiddle W_48^{(j%3) q},
//             outputs rows 48 g + j%3 + 3 q;
//   stage 3:  radix-16 butterfly j (Ns = 48): rows j + 48 q, twiddle
//             W_768^{j q}, natural-order outputs k1 = j + 48 q stored to global
//             with W_M^{n' k1} (exact at q = 0 and 8, stepped in between).
__global__ void __launch_bounds__(kThrA) colA_kernel(ColAArgs a) {
  __shared__ __attribute__((aligned(16))) float2 data[kL1 * kCols];
  __shared__ float2 w768[kL1];
  __shared__ float lut_s[kLutSize], lut_c[kLutSize];
  __shared__ double red[kThrA / kWave + 1];

  const int b = blockIdx.y;
  const uint32_t col0 = blockIdx.x * kCols;
  const int c = threadIdx.x % kCols;
  const int j = threadIdx.x / kCols;
  const uint32_t ncol = col0 + c;  // n'
  if (a.reset != nullptr && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) *a.reset = 0;

  for (int i = threadIdx.x; i < kLutSize; i += kThrA) {
    lut_s[i] = kSinLut[i];
    lut_c[i] = kCosLut[i];
  }
  for (int e = threadIdx.x; e < kL1; e += kThrA) w768[e] = a.w768[e];
  __syncthreads();

  // gather (three phases: all indices, all loads, then centre + store)
  constexpr int kRowsData = kL1 / 3;                      // 256
  constexpr int kU = (kRowsData + 47) / 48;               // 6 row iterations
  const bool fast = a.n_unpadded <= (1u << 23);
  const TemplateDev td = a.tmpl[b];
  const float* series = a.series + static_cast<size_t>(td.wu) * a.n_unpadded;
  const int last = static_cast<int>(a.n_unpadded) - 1;
  int idx[2 * kU];
#pragma unroll
  for (int u = 0; u < kU; ++u) {
    const int r = j + 48 * u;
    const uint32_t m0 = 2 * (static_cast<uint32_t>(r) * kR + ncol);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint32_t m = m0 + h;
      int i = -1;
      if (r < kRowsData && m < td.n_steps) {
        const float dt = resamp_del_t(m, td.p, lut_s, lut_c);
        i = min(max(fast ? resamp_nearest_f(m, dt) : resamp_nearest(m, dt), 0), last);
      }
      idx[2 * u + h] = i;
    }
  }
  float raw[2 * kU];
#pragma unroll
  for (int e = 0; e < 2 * kU; ++e) raw[e] = series[idx[e] < 0 ? 0 : idx[e]];
  float fsum = 0.0f;
#pragma unroll
  for (int u = 0; u < kU; ++u) {
    const int r = j + 48 * u;
    const float x0 = idx[2 * u] < 0 ? 0.0f : raw[2 * u] - td.mu0;
    const float x1 = idx[2 * u + 1] < 0 ? 0.0f : raw[2 * u + 1] - td.mu0;
    fsum += x0 + x1;
    if (r < kRowsData) data[r * kCols + c] = make_float2(x0, x1);
  }
  __syncthreads();

  // stages 1 + 2
  {
    const int g = j / 3, s = j % 3;
    float2 y[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) y[q] = data[(g + 16 * q) * kCols + c];
    if (s != 0) {
#pragma unroll
      for (int q = 1; q < 16; ++q) y[q] = cmul(y[q], w768[(16 * s * q) % kL1]);
    }
    Dft<16>::run(y);
    __syncthreads();  // all inputs read before the in-place scatter
#pragma unroll
    for (int q = 0; q < 16; ++q) data[(48 * g + s + 3 * q) * kCols + c] = y[q];
  }
  __syncthreads();

  // stage 3 + store
  {
    float2 z[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) z[q] = data[(j + 48 * q) * kCols + c];
#pragma unroll
    for (int q = 1; q < 16; ++q) z[q] = cmul(z[q], w768[j * q]);
    Dft<16>::run(z);
    // W_M^{n' k1} = W_4M^{4 n' k1}
    const uint64_t p4 = a.tw.period;
    const float2 step = tw_lookup(a.tw, (4ull * ncol * 48u) % p4);
    float2 t0 = tw_lookup(a.tw, (4ull * ncol * static_cast<uint32_t>(j)) % p4);
    float2 t8 = tw_lookup(a.tw, (4ull * ncol * static_cast<uint32_t>(j + 48 * 8)) % p4);
    float2* out = a.out + static_cast<size_t>(b) * a.M + ncol;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      out[static_cast<size_t>(j + 48 * q) * kR] = cmul(z[q], t0);
      out[static_cast<size_t>(j + 48 * (q + 8)) * kR] = cmul(z[q + 8], t8);
      t0 = cmul(t0, step);
      t8 = cmul(t8, step);
    }
  }
  const double tot = block_sum<kThrA>(static_cast<double>(fsum), red);
  if (threadIdx.x == 0) a.partials[static_cast<size_t>(b) * gridDim.x + blockIdx.x] = tot;
}

// ------------------------------------------------------------------ pass B
// Row layout with one pad element every 16 (bank spreading of the stride-16
// Stockham scatters); pitch == 16 (mod 32).
constexpr int kPitchB = row_pitch<kR>();
__device__ __forceinline__ int bidx(int r, int slot) { return slot * kPitchB + r + (r >> 4); }

// One radix-16 Stockham stage of both rows, LDS -> LDS. Thread (slot, j)
// owns butterfly j < 512 of its row; twiddle W_{16 Ns}^{(j mod Ns) q} = tw(e).
template <int NS, typename TwF>
__device__ __forceinline__ void rowB_stage16(float2* lds, int slot, int j, TwF tw) {
  float2 v[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) v[q] = lds[bidx(j + 512 * q, slot)];
  const int jm = j % NS;
#pragma unroll
  for (int q = 1; q < 16; ++q) v[q] = cmul(v[q], tw(jm * q));
  Dft<16>::run(v);
  __syncthreads();
  const int base = (j / NS) * NS * 16 + jm;
#pragma unroll
  for (int q = 0; q < 16; ++q) lds[bidx(base + q * NS, slot)] = v[q];
  __syncthreads();
}

// One workgroup per row pair (140 KB of LDS: one workgroup per CU). A
// persistent variant that prefetches the next pair into registers was
// measured slower (46.7 vs 35 us/template: the prefetch registers spill).
__global__ void __launch_bounds__(kThrB) rowB_kernel(RowBArgs a) {
  __shared__ __attribute__((aligned(16))) float2 data[2 * kPitchB];
  __shared__ float2 t256[256];           // W_256^e
  __shared__ float2 t4096[128];          // W_4096: lo[64] | hi[64] (step 64)
  __shared__ float2 t8192[128];          // W_8192: lo[64] | hi[64] (step 64), e < 4096
  __shared__ double red[kThrB / kWave + 1];

  const int b = blockIdx.y;
  const uint32_t k1 = blockIdx.x;                      // 0 .. L1/2
  const uint32_t k1m = (kL1 - k1) % kL1;               // mirror row
  const int slot = threadIdx.x / 512;
  const int j = threadIdx.x % 512;

  // stage 1 (radix 16, Ns = 1) straight from global: elements j + 512 q
  {
    const float2* src = a.buf + static_cast<size_t>(b) * a.M + static_cast<size_t>(slot ? k1m : k1) * kR;
    float2 v[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) v[q] = src[j + 512 * q];
    for (int e = threadIdx.x; e < 256; e += kThrB) t256[e] = a.t256[e];
    for (int e = threadIdx.x; e < 128; e += kThrB) {
      t4096[e] = a.t4096[e];
      t8192[e] = a.t8192[e];
    }
    Dft<16>::run(v);
#pragma unroll
    for (int q = 0; q < 16; ++q) data[bidx(16 * j + q, slot)] = v[q];
  }
  // mean-padding correction: delta = sum(partials) / n_steps, same fixed order in every workgroup
  const uint32_t n_s = a.tmpl[b].n_steps;
  double part = 0.0;
  for (uint32_t i = threadIdx.x; i < a.n_partials; i += kThrB) part += a.partials[static_cast<size_t>(b) * a.n_partials + i];
  const double tot = block_sum<kThrB>(part, red);  // (its barriers also publish stage 1)
  const float dS = n_s ? static_cast<float>(tot / static_cast<double>(n_s)) : 0.0f;

  rowB_stage16<16>(data, slot, j, [&](int e) { return t256[e]; });
  rowB_stage16<256>(data, slot, j, [&](int e) { return cmul(t4096[64 + (e >> 6)], t4096[e & 63]); });

  // stage 4 (radix 2, Ns = 4096) fused with the untangle. Thread t owns
  // butterflies jj = t + 1024 u (u < 4) of row k1 (outputs m = jj, jj + 4096)
  // and butterfly jm = 4095 - jj of the mirror row (outputs R-1-jj-4096 and
  // R-1-jj): together the four partners of two untangle pairs. Row 0 pairs
  // with itself shifted by one (m <-> R - m): butterfly (4096 - jj) % 4096.
  const int t = threadIdx.x;
  const bool row0 = (k1 == 0);
  const bool self = row0 || (k1 == kL1 / 2);  // mirror row == row: emit only bins of row k1
  const bool correct = n_s > 0;
  float* pss = a.pss + static_cast<size_t>(b) * a.pss_stride;
  auto w8192 = [&](int e) { return cmul(t8192[64 + (e >> 6)], t8192[e & 63]); };
  auto emit = [&](uint32_t row, uint32_t m, float2 x, float2 tk, float2 ta) {
    const uint32_t k = row + kL1 * m;
    if (k >= a.limit) return;
    float p = 0.0f;
    if (k != 0) {
      if (correct) {
        const float ratio = ta.y * __builtin_amdgcn_rcpf(tk.y);
        const float2 tc = cmul(ta, conjf2(tk));  // W_2N^{(n_s-1) k}
        x = make_float2(x.x - dS * ratio * tc.x, x.y - dS * ratio * tc.y);
      }
      p = (x.x * x.x + x.y * x.y) * a.norm;
    }
    pss[row * kR + m] = p;
  };
  // bin M - k = k1m + L1 (R - 1 - m): W_N^{M-k} = -conj(W_N^k),
  // W_2N^{M-k} = -i conj(W_2N^k), W_2N^{n_s (M-k)} = (-i)^{n_s} conj(W_2N^{n_s k})
  auto emit_pair = [&](uint32_t m, float2 zk, float2 zm, float2 tk, float2 ta) {
    const float2 w = cmul(tk, tk);  // W_N^k
    emit(k1, m, untangle_w(zk, zm, w), tk, ta);
    if (!self) emit(k1m, kR - 1 - m, untangle_w(zm, zk, make_float2(-w.x, w.y)), make_float2(-tk.y, -tk.x),
                    rot_mi(conjf2(ta), n_s));
  };
  // twiddles of bin k = k1 + L1 m for m = t + 1024 u (A) and m + 4096 (B):
  // W_2N^k and W_2N^{n_s k}, stepped by W_2N^{1024 L1} and W_2N^{1024 L1 n_s}
  const uint64_t P = a.tw.period;
  const uint64_t ka = (k1 + static_cast<uint64_t>(kL1) * t) % P;
  const uint64_t kb = (k1 + static_cast<uint64_t>(kL1) * (t + 4096)) % P;
  float2 tkA = tw_lookup(a.tw, ka), tkB = tw_lookup(a.tw, kb);
  const float2 tk_step = tw_lookup(a.tw, (1024ull * kL1) % P);
  float2 taA = make_float2(1.f, 0.f), taB = taA, ta_step = taA;
  if (correct) {
    taA = tw_lookup(a.tw, (static_cast<uint64_t>(n_s) * ka) % P);
    taB = tw_lookup(a.tw, (static_cast<uint64_t>(n_s) * kb) % P);
    ta_step = tw_lookup(a.tw, (static_cast<uint64_t>(n_s) * ((1024ull * kL1) % P)) % P);
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int jj = t + 1024 * u;
    const float2 x0 = data[bidx(jj, 0)], x1 = cmul(data[bidx(jj + 4096, 0)], w8192(jj));
    const float2 zlo = cadd(x0, x1), zhi = csub(x0, x1);
    const int jm = row0 ? (4096 - jj) % 4096 : 4095 - jj;
    const float2 y0 = data[bidx(jm, 1)], y1 = cmul(data[bidx(jm + 4096, 1)], w8192(jm));
    const float2 lo = cadd(y0, y1), hi = csub(y0, y1);  // mirror m = jm, jm + 4096
    // partner of m = jj: R-1-jj (= jm + 4096) in general, (R - jj) % R for row 0
    const bool r00 = row0 && jj == 0;
    const float2 mlo = r00 ? lo : hi, mhi = r00 ? hi : lo;
    if (u > 0) {
      tkA = cmul(tkA, tk_step);
      tkB = cmul(tkB, tk_step);
      if (correct) {
        taA = cmul(taA, ta_step);
        taB = cmul(taB, ta_step);
      }
    }
    emit_pair(static_cast<uint32_t>(jj), zlo, mlo, tkA, taA);
    emit_pair(static_cast<uint32_t>(jj + 4096), zhi, mhi, tkB, taB);
    if (row0 && jj == 0 && a.M < a.limit) {
      // Nyquist bin M = L1 R: X_M = Re Z_0 - Im Z_0 (written in natural order)
      float2 x = make_float2(zlo.x - zlo.y, 0.0f);
      if (correct) {
        const float2 tkM = tw_lookup(a.tw, a.M % P), taM = tw_lookup(a.tw, (static_cast<uint64_t>(n_s) * a.M) % P);
        const float2 sp = padding_spectrum_t(taM, tkM, cmul(taM, conjf2(tkM)));
        x = make_float2(x.x + dS * sp.x, x.y + dS * sp.y);
      }
      const float pm = (x.x * x.x + x.y * x.y) * a.norm;
      if (a.ps16) a.ps16[static_cast<size_t>(b) * a.ps_stride + a.M] = static_cast<_Float16>(pm);
      else a.ps[static_cast<size_t>(b) * a.ps_stride + a.M] = pm;
    }
  }
}

// -------------------------------------------------------------- transpose
// PS[k] = PSs[k % L1][k / L1] for k < min(limit, M); 64 x 64 tiles via LDS.
template <bool HALF>
__global__ void __launch_bounds__(256) psT_kernel(PsTArgs a) {
  __shared__ float tile[64][65];
  const int b = blockIdx.z;
  const uint32_t r0 = blockIdx.x * 64;  // k1
  const uint32_t m0 = blockIdx.y * 64;  // m
  const float* src = a.pss + static_cast<size_t>(b) * a.pss_stride;
  const int tx = threadIdx.x % 16, ty = threadIdx.x / 16;
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int r = ty + 16 * rr;
    const float4 v = *reinterpret_cast<const float4*>(src + static_cast<size_t>(r0 + r) * kR + m0 + 4 * tx);
    tile[r][4 * tx + 0] = v.x;
    tile[r][4 * tx + 1] = v.y;
    tile[r][4 * tx + 2] = v.z;
    tile[r][4 * tx + 3] = v.w;
  }
  __syncthreads();
  const uint32_t kmax = a.limit < a.M ? a.limit : a.M;
  const int lane = threadIdx.x % 64, w = threadIdx.x / 64;
#pragma unroll
  for (int mm = 0; mm < 16; ++mm) {
    const int m = w + 4 * mm;
    const uint32_t k = r0 + lane + kL1 * (m0 + m);
    if (k < kmax) {
      const float v = tile[lane][m];
      if (HALF) a.ps16[static_cast<size_t>(b) * a.ps_stride + k] = static_cast<_Float16>(v);
      else a.ps[static_cast<size_t>(b) * a.ps_stride + k] = v;
    }
  }
}

}  // namespace

hipError_t launch_colA(const ColAArgs& a, int batch, hipStream_t s) {
  hipLaunchKernelGGL(colA_kernel, dim3(kR / kCols, batch), dim3(kThrA), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_rowB(const RowBArgs& a, int batch, hipStream_t s) {
  hipLaunchKernelGGL(rowB_kernel, dim3(kL1 / 2 + 1, batch), dim3(kThrB), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_psT(const PsTArgs& a, int batch, hipStream_t s) {
  const uint32_t kmax = std::min(a.limit, a.M);
  const uint32_t mrows = (kmax + kL1 - 1) / kL1;  // m < mrows hold bins < kmax
  const dim3 grid(kL1 / 64, (mrows + 63) / 64, batch);
  if (a.ps16) hipLaunchKernelGGL(psT_kernel<true>, grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL(psT_kernel<false>, grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace hipk
}  // namespace brp
