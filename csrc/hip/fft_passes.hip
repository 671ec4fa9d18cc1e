// Three-pass packed real FFT for gfx950 with fused prologue/epilogue:
//   pass 1: nearest-neighbour resampling gather (or real / complex load) fused
//           into the load of L1-point column FFTs
//   pass 2: L2-point column FFTs, in place
//   pass 3: L3-point row FFTs + real-FFT untangle + normalised power spectrum
//           (+ analytic mean-padding correction), natural-order output
// See fft_plan.hpp for the index algebra. Replaces the reference's cuFFT /
// clFFT / FFTW calls (cuda/app/demod_binary_cuda.cu:849-965,
// opencl/app/demod_binary_ocl.cpp:972-1314, demod_binary_fft_fftw.c:46-113) and
// its resampling kernels (cuda/app/demod_binary_cuda.cuh:69-184).
#include <algorithm>
#include <type_traits>

#include "bluestein_kernels.hpp"
#include "fft_block.hpp"
#include "fft_kernels.hpp"

namespace brp {
namespace hipk {

namespace {

constexpr int kNcol = 16;

template <int L>
constexpr int tpc_for() {
  return (L / 16) < 1 ? 1 : (L / 16);
}

// ------------------------------------------------------------------ pass 1
template <int L, int MODE>
__global__ void __launch_bounds__(kNcol * tpc_for<L>()) pass1_kernel(Pass1Args a) {
  constexpr int TPC = tpc_for<L>();
  constexpr int NT = kNcol * TPC;
  using Lay = BlockLayout<L, kNcol, TPC, false>;
  // data | stage twiddles W_L | output twiddles W_{L1 L2}^{n2 k1} | reduction scratch
  __shared__ __attribute__((aligned(16))) float2 smem[Lay::kLds + kTwPad<L> + L + 16];
  float2* data = smem;
  float2* twl = smem + Lay::kLds;
  float2* two = twl + kTwPad<L>;
  double* red = reinterpret_cast<double*>(two + L);

  const int b = blockIdx.y;
  const uint32_t nblk3 = a.L3 / kNcol;
  const uint32_t n2 = blockIdx.x / nblk3;
  const uint32_t col_base = n2 * a.L3 + (blockIdx.x % nblk3) * kNcol;
  const size_t M = static_cast<size_t>(L) * a.L2L3;

  int c, tj;
  Lay::coords(threadIdx.x, c, tj);
  if (a.reset != nullptr && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) BRP_ST(a.reset, 0u);

  double sum = 0.0, sum_b = 0.0;  // sum_b: the second template of a pair (P1_CHIRP1_PAIR)
  bool pruned = false;
  if (MODE == P1_RESAMPLE) {
    __shared__ float lut_s[kLutSize], lut_c[kLutSize];
    for (int i = threadIdx.x; i < kLutSize; i += NT) {
      lut_s[i] = kSinLut[i];
      lut_c[i] = kCosLut[i];
    }
    __syncthreads();
    const bool fast = a.n_unpadded <= (1u << 23);
    const TemplateDev td = BRP_LD(&a.tmpl[b]);
    const float* series = a.series + static_cast<size_t>(td.wu) * a.n_unpadded;
    // With padding >= R0 (the first radix) every row n1 >= L/R0 of the
    // tile lies in the zero padding: those rows are neither resampled nor
    // stored, and the FFT's first stage replicates (BlockFFT::run_pruned).
    constexpr int kR0 = BlockFFT<L, kNcol, TPC, false>::kFirstRadix;
    pruned = 2ull * (L / kR0) * a.L2L3 >= td.n_steps;
    // three phases so that all gathers of the thread are in flight together:
    // nearest indices (LUT sine, VALU), unconditional clamped loads, then
    // select/centre/accumulate into LDS. NU = row iterations of the thread
    // (all L rows, or the L/R0 rows outside the padding).
    const int last = static_cast<int>(a.n_unpadded) - 1;
    const int rows_valid = pruned ? L / kR0 : L;
    auto gather = [&](auto nu_tag) {
      constexpr int NU = decltype(nu_tag)::value;
      constexpr int ROWS = NU * TPC;
      int idx[2 * NU];
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const int r = tj + u * TPC;
        const uint32_t m0 = 2 * (r * a.L2L3 + col_base + c);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const uint32_t m = m0 + q;
          int i = -1;
          if ((ROWS == L || r < rows_valid) && m < td.n_steps) {
            const float dt = resamp_del_t(m, td.p, lut_s, lut_c);
            i = min(max(fast ? resamp_nearest_f(m, dt) : resamp_nearest(m, dt), 0), last);
          }
          idx[2 * u + q] = i;
        }
      }
      float raw[2 * NU];
#pragma unroll
      for (int e = 0; e < 2 * NU; ++e) raw[e] = BRP_LD(&series[idx[e] < 0 ? 0 : idx[e]]);
      // per-thread partial sum in float, widened once for the block reduction
      float fsum = 0.0f;
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const int r = tj + u * TPC;
        const float x0 = idx[2 * u] < 0 ? 0.0f : raw[2 * u] - td.mu0;
        const float x1 = idx[2 * u + 1] < 0 ? 0.0f : raw[2 * u + 1] - td.mu0;
        fsum += x0 + x1;
        if (ROWS == L || r < rows_valid) data[Lay::idx(r, c)] = make_float2(x0, x1);
      }
      return fsum;
    };
    constexpr int kPer = L / TPC;
    constexpr int kPerPruned = (L / kR0 + TPC - 1) / TPC;
    const float fsum = pruned ? gather(std::integral_constant<int, kPerPruned>{})
                              : gather(std::integral_constant<int, kPer>{});
    sum = static_cast<double>(fsum);
  } else if (MODE == P1_CHIRP2 || MODE == P1_CHIRP1 || MODE == P1_CHIRP1_PAIR) {
    __shared__ float lut_s[kLutSize], lut_c[kLutSize];
    for (int i = threadIdx.x; i < kLutSize; i += NT) {
      lut_s[i] = kSinLut[i];
      lut_c[i] = kCosLut[i];
    }
    __syncthreads();
    constexpr bool kPair = MODE == P1_CHIRP1_PAIR;
    const bool fast = a.n_unpadded <= (1u << 23);
    const int ta = kPair ? 2 * b : b;
    const bool has_b = kPair && static_cast<uint32_t>(ta + 1) < a.n_tmpl;
    const TemplateDev td = BRP_LD(&a.tmpl[ta]);
    TemplateDev tdb = td;
    if (has_b) tdb = BRP_LD(&a.tmpl[ta + 1]);
    const float* series = a.series + static_cast<size_t>(td.wu) * a.n_unpadded;
    const float* series_b = a.series + static_cast<size_t>(tdb.wu) * a.n_unpadded;
    const int last = static_cast<int>(a.n_unpadded) - 1;
    // the convolution input is zero from Mb on (L >= 2 Mb - 1): with
    // Mb <= (L / R0) L2L3 the rows n1 >= L / R0 are all zero (run_pruned)
    constexpr int kR0 = BlockFFT<L, kNcol, TPC, false>::kFirstRadix;
    pruned = static_cast<uint64_t>(L / kR0) * a.L2L3 >= a.Mb;
    const int rows_valid = pruned ? L / kR0 : L;
    auto sample_of = [&](const TemplateDev& t, const float* ser, uint32_t m) -> float {
      if (m >= t.n_steps) return 0.0f;
      const float dt = resamp_del_t(m, t.p, lut_s, lut_c);
      const int i = min(max(fast ? resamp_nearest_f(m, dt) : resamp_nearest(m, dt), 0), last);
      return BRP_LD(&ser[i]) - t.mu0;
    };
    auto sample = [&](uint32_t m) { return sample_of(td, series, m); };
    float fsum = 0.0f, fsum_b = 0.0f;
    for (int r = tj; r < rows_valid; r += TPC) {
      const uint32_t n = r * a.L2L3 + col_base + c;
      float2 v = make_float2(0.0f, 0.0f);
      if (n < a.Mb) {
        float2 x;
        if (MODE == P1_CHIRP2) {
          x = make_float2(sample(2 * n), sample(2 * n + 1));
          fsum += x.x + x.y;
        } else {
          x = make_float2(sample(n), has_b ? sample_of(tdb, series_b, n) : 0.0f);
          fsum += x.x;
          fsum_b += x.y;
        }
        v = cmul(x, tw_lookup(a.chirp, static_cast<uint64_t>(n) * n));  // W_{2Mb}^{n^2 mod 2Mb}
      }
      data[Lay::idx(r, c)] = v;
    }
    sum = static_cast<double>(fsum);
    sum_b = static_cast<double>(fsum_b);
  } else if (MODE == P1_REAL) {
    for (int r = tj; r < L; r += TPC) {
      const uint32_t n = r * a.L2L3 + col_base + c;
      const float x0 = (2 * n < a.n_real) ? BRP_LD(&a.real_in[2 * n]) : 0.0f;
      const float x1 = (2 * n + 1 < a.n_real) ? BRP_LD(&a.real_in[2 * n + 1]) : 0.0f;
      data[Lay::idx(r, c)] = make_float2(x0, x1);
    }
  } else {
    for (int r = tj; r < L; r += TPC) {
      const uint32_t n = r * a.L2L3 + col_base + c;
      const float2 v = BRP_LD(&a.cplx_in[static_cast<size_t>(b) * M + n]);
      data[Lay::idx(r, c)] = MODE == P1_COMPLEX_CONJ ? conjf2(v) : v;
    }
  }
  copy_stage_twiddles<L>(twl, a.tb.st1);
  for (int k1 = threadIdx.x; k1 < L; k1 += NT) two[k1] = BRP_LD(&a.tb.p1[n2 * L + k1]);  // W_{L1 L2}^{n2 k1}
  __syncthreads();
  if (pruned) BlockFFT<L, kNcol, TPC, false>::run_pruned(data, twl);
  else BlockFFT<L, kNcol, TPC, false>::run(data, twl);

  float2* out = a.out + static_cast<size_t>(b) * M;
  for (int k1 = tj; k1 < L; k1 += TPC) {
    const float2 v = cmul(data[Lay::idx(k1, c)], two[k1]);
    BRP_ST(&out[static_cast<size_t>(k1) * a.L2L3 + col_base + c], v);
  }
  if (MODE == P1_RESAMPLE || MODE == P1_CHIRP2 || MODE == P1_CHIRP1) {
    const double tot = block_sum<NT>(sum, red);
    if (threadIdx.x == 0) BRP_ST(&a.partials[static_cast<size_t>(b) * gridDim.x + blockIdx.x], tot);
  } else if (MODE == P1_CHIRP1_PAIR) {  // partial sums per template (2b, 2b + 1)
    const double tot = block_sum<NT>(sum, red);
    const double tot_b = block_sum<NT>(sum_b, red);
    if (threadIdx.x == 0) {
      BRP_ST(&a.partials[static_cast<size_t>(2 * b) * gridDim.x + blockIdx.x], tot);
      if (static_cast<uint32_t>(2 * b + 1) < a.n_tmpl)
        BRP_ST(&a.partials[static_cast<size_t>(2 * b + 1) * gridDim.x + blockIdx.x], tot_b);
    }
  }
}

// Resampling pass 1 for L = 3 * R2 * 16 when the padding is at least 3x
// (every row n1 >= L/3 of a column lies in the zero padding). Stage 1 (radix
// 3 on rows that are zero beyond L/3) replicates, so stage 1 + stage 2 (radix
// R2, Ns = 3) of butterfly group g = j/3 read only the gathered rows
// g + 16 q (q < R2) and produce rows 12 g .. 12 g + 3 R2 - 1: one thread per
// group gathers exactly its inputs and computes the three radix-R2
// butterflies in registers. The tile crosses LDS once; the last stage (radix
// 16, Ns = 3 R2) stores its natural-order rows k1 = j + 3 R2 q straight to
// global memory with the output twiddle W_{L1 L2}^{n2 k1}.
// Speed-of-light ablations for experiment builds (scripts/build_variant.sh,
// wrong results): BRP_ABLATE_P1FFT / P1RES drop pass 1's butterflies / its
// resampling arithmetic, BRP_ABLATE_P3FFT pass 3's row FFT; the memory
// traffic of every pass is unchanged.
#ifdef BRP_ABLATE_P1FFT
constexpr bool kAblateP1Fft = true;
#else
constexpr bool kAblateP1Fft = false;
#endif
#ifdef BRP_ABLATE_P1RES
constexpr bool kAblateP1Res = true;
#else
constexpr bool kAblateP1Res = false;
#endif
#ifdef BRP_ABLATE_P3FFT
constexpr bool kAblateP3Fft = true;
#else
constexpr bool kAblateP3Fft = false;
#endif

#ifndef BRP_P1_WAVES
#define BRP_P1_WAVES 4  // waves per SIMD the register budget allows (build switch; 5 spills 24 B)
#endif
template <int R2>
__global__ void __launch_bounds__(kNcol * 16) __attribute__((amdgpu_waves_per_eu(BRP_P1_WAVES, 8)))
pass1_pruned3_kernel(Pass1Args a) {
  constexpr int L = 3 * R2 * 16;
  constexpr int TPC = 16;               // threads per column = butterfly groups of stages 1+2
  constexpr int NT = kNcol * TPC;
  constexpr int NB3 = 3 * R2;           // last-stage butterflies per column (threads tj < NB3)
  static_assert(NB3 <= TPC, "one last-stage butterfly per thread");
  __shared__ __attribute__((aligned(16))) float2 data[L * kNcol];
  __shared__ float2 wl[L];              // W_L^e
  __shared__ float2 two[L];             // W_{L1 L2}^{n2 k1}
  __shared__ float lut_s[kLutSize], lut_c[kLutSize];
  __shared__ double red[NT / kWave + 1];

  const int b = blockIdx.y;
  const uint32_t nblk3 = a.L3 / kNcol;
  const uint32_t n2 = blockIdx.x / nblk3;
  const uint32_t col_base = n2 * a.L3 + (blockIdx.x % nblk3) * kNcol;
  const size_t M = static_cast<size_t>(L) * a.L2L3;
  const int c = threadIdx.x % kNcol;
  const int tj = threadIdx.x / kNcol;
  if (a.reset != nullptr && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) BRP_ST(a.reset, 0u);

  // the template, the sine LUT and the twiddle tables are loaded together
  // before the first LDS write (one memory round trip instead of three ahead
  // of the gather)
  static_assert(kLutSize <= NT && L <= NT, "one LUT / table entry per thread");
  const TemplateDev td = BRP_LD(&a.tmpl[b]);
  const int tid = static_cast<int>(threadIdx.x);
  float ls = 0.0f, lc = 0.0f;
  float2 wv = make_float2(0.0f, 0.0f), tv = wv;
  if (tid < kLutSize) {
    ls = kSinLut[tid];
    lc = kCosLut[tid];
  }
  if (tid < L) {
    wv = BRP_LD(&a.tb.st1[tid + (tid >> 4)]);
    tv = BRP_LD(&a.tb.p1[n2 * L + tid]);
  }
  if (tid < kLutSize) {
    lut_s[tid] = ls;
    lut_c[tid] = lc;
  }
  if (tid < L) {
    wl[tid] = wv;
    two[tid] = tv;
  }
  __syncthreads();

  // gather rows g + 16 q (q < R2) of column c: nearest-neighbour resampling
  // with the reference's float arithmetic (three phases keep all loads in flight)
  const bool fast = a.n_unpadded <= (1u << 23);
  const float* series = a.series + static_cast<size_t>(td.wu) * a.n_unpadded;
  const int last = static_cast<int>(a.n_unpadded) - 1;
  int idx[2 * R2];
#pragma unroll
  for (int q = 0; q < R2; ++q) {
    const uint32_t m0 = 2 * ((tj + 16 * q) * a.L2L3 + col_base + c);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint32_t m = m0 + h;
      int i = -1;
      if (m < td.n_steps) {
        if constexpr (kAblateP1Res) {
          i = min(static_cast<int>(m), last);
        } else {
          const float dt = resamp_del_t(m, td.p, lut_s, lut_c);
          i = min(max(fast ? resamp_nearest_f(m, dt) : resamp_nearest(m, dt), 0), last);
        }
      }
      idx[2 * q + h] = i;
    }
  }
  float raw[2 * R2];
#pragma unroll
  for (int e = 0; e < 2 * R2; ++e)
    raw[e] = BRP_LD(&series[BRP_INJECT_AT(idx[e] < 0 ? 0 : idx[e], last + 17, kInjPass1)]);
  float fsum = 0.0f;
  float2 x[R2];
#pragma unroll
  for (int q = 0; q < R2; ++q) {
    const float x0 = idx[2 * q] < 0 ? 0.0f : raw[2 * q] - td.mu0;
    const float x1 = idx[2 * q + 1] < 0 ? 0.0f : raw[2 * q + 1] - td.mu0;
    fsum += x0 + x1;
    x[q] = make_float2(x0, x1);
  }
  // stages 1+2: butterfly j = 3 tj + s (s < 3) is a radix-R2 DFT of the
  // group's rows with twiddle W_{3 R2}^{s q} = W_L^{16 s q}; its outputs
  // are rows 12 tj + s + 3 q
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    float2 y[R2];
#pragma unroll
    for (int q = 0; q < R2; ++q) y[q] = (s == 0 || q == 0) ? x[q] : cmul(x[q], wl[(16 * s * q) % L]);
    if constexpr (!kAblateP1Fft) Dft<R2>::run(y);
#pragma unroll
    for (int q = 0; q < R2; ++q) data[(NB3 * tj + s + 3 * q) * kNcol + c] = y[q];
  }
  __syncthreads();
  // stage 3 (radix 16, Ns = 3 R2): butterfly j = tj reads rows j + NB3 q
  if (tj < NB3) {
    float2 z[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) z[q] = lds_ld64(&data[(tj + NB3 * q) * kNcol + c]);  // b64, not read2
#pragma unroll
    for (int q = 1; q < 16; ++q) z[q] = cmul(z[q], wl[tj * q]);
    if constexpr (!kAblateP1Fft) Dft<16>::run(z);
    float2* out = a.out + static_cast<size_t>(b) * M + col_base + c;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int k1 = tj + NB3 * q;
      BRP_ST(&out[static_cast<size_t>(k1) * a.L2L3], cmul(z[q], lds_ld64(&two[k1])));
    }
  }
  const double tot = block_sum<NT>(static_cast<double>(fsum), red);
  if (threadIdx.x == 0) BRP_ST(&a.partials[static_cast<size_t>(b) * gridDim.x + blockIdx.x], tot);
}

// ------------------------------------------------------------------ pass 2
// mean-padding correction of the templates of transform b (one, or two for
// paired chirp-z transforms), each reduced once in a fixed order:
// delta[t] = (sum of pass 1's partial sums of template t) / n_steps
template <int NT>
__device__ __forceinline__ void reduce_delta(const Pass2Args& a, uint32_t b, double* red) {
  const uint32_t tpt = a.tpt > 1 ? a.tpt : 1;
  for (uint32_t q = 0; q < tpt; ++q) {
    const uint32_t t = b * tpt + q;
    if (tpt > 1 && t >= a.n_tmpl) break;  // uniform
    const double* pp = a.partials + static_cast<size_t>(t) * a.n_partials;
    double part = 0.0;
    for (uint32_t i = threadIdx.x; i < a.n_partials; i += NT) part += BRP_LD(&pp[i]);
    const double tot = block_sum<NT>(part, red);
    if (threadIdx.x == 0) {
      const uint32_t n_s = BRP_LD(&a.tmpl[t]).n_steps;
      BRP_ST(&a.delta[t], n_s ? tot / static_cast<double>(n_s) : 0.0);
    }
  }
}

// at least kMinWaves waves per SIMD: keeps the unrolled prefetch + FFT code
// within 256 VGPRs (no spills) at 2 waves/SIMD
constexpr int kMinWaves = 2;

constexpr int kP2LoBits = 8;

// Persistent: each workgroup walks tiles (template b, column k1, 16 columns n3)
// blockIdx.x, +gridDim.x, ...; the next tile's columns are loaded into
// registers while the current one is transformed and stored, and the fixed
// twiddle tables are staged in LDS once per workgroup.
template <int L>
__global__ void __launch_bounds__(kNcol * tpc_for<L>(), kMinWaves) pass2_kernel(Pass2Args a, uint32_t ntiles) {
  constexpr int TPC = tpc_for<L>();
  constexpr int NT = kNcol * TPC;
  constexpr int kPer = L / TPC;
  using Lay = BlockLayout<L, kNcol, TPC, false>;
  constexpr int kLo = 1 << kP2LoBits;
  constexpr int kHiMax = 1024;  // L2*L3 <= 2^18
  // data | stage twiddles | W_{L2L3} lo | W_{L2L3} hi
  __shared__ __attribute__((aligned(16))) float2 smem[Lay::kLds + kTwPad<L> + kLo + kHiMax];
  __shared__ double red[NT / kWave + 1];
  float2* data = smem;
  float2* twl = smem + Lay::kLds;
  float2* lo = twl + kTwPad<L>;
  float2* hi = lo + kLo;

  const uint32_t nblk3 = a.L3 / kNcol;
  const uint32_t per_b = a.L1 * nblk3;
  const size_t M = static_cast<size_t>(a.L1) * a.L2L3;
  int c, tj;
  Lay::coords(threadIdx.x, c, tj);
  auto tile_base = [&](uint32_t tl) -> size_t {
    const uint32_t b = tl / per_b, rem = tl % per_b;
    return static_cast<size_t>(b) * M + static_cast<size_t>(rem / nblk3) * a.L2L3 + (rem % nblk3) * kNcol;
  };

  float2 pre[kPer];
  uint32_t tile = blockIdx.x;
  if (tile < ntiles) {
    const float2* src = a.buf + tile_base(tile);
#pragma unroll
    for (int u = 0; u < kPer; ++u) pre[u] = BRP_LD(&src[static_cast<size_t>(tj + u * TPC) * a.L3 + c]);
  }
  {
    copy_stage_twiddles<L>(twl, a.tb.st2);
    const uint32_t nhi = (a.L2L3 + kLo - 1) / kLo;
    for (int i = threadIdx.x; i < kLo; i += NT) lo[i] = BRP_LD(&a.tb.p2lo[i]);
    for (uint32_t i = threadIdx.x; i < nhi; i += NT) hi[i] = BRP_LD(&a.tb.p2hi[i]);
  }
  while (tile < ntiles) {
    const uint32_t b = tile / per_b, rem = tile % per_b;
    const uint32_t k1 = rem / nblk3;
    const uint32_t n3 = (rem % nblk3) * kNcol + c;
    float2* base = a.buf + tile_base(tile);
#pragma unroll
    for (int u = 0; u < kPer; ++u) data[Lay::idx(tj + u * TPC, c)] = pre[u];
    // W_M^{n3 (k1 + L1 k2)} = W_M^{n3 k1} * W_{L2 L3}^{n3 k2}
    const float2 wc = BRP_LD(&a.tb.p2col[k1 * a.L3 + n3]);
    const uint32_t next = tile + gridDim.x;
    if (next < ntiles) {  // in flight during this tile's FFT and stores
      const float2* src = a.buf + tile_base(next);
#pragma unroll
      for (int u = 0; u < kPer; ++u) pre[u] = BRP_LD(&src[static_cast<size_t>(tj + u * TPC) * a.L3 + c]);
    }
    __syncthreads();
    BlockFFT<L, kNcol, TPC, false>::run(data, twl);
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int k2 = tj + u * TPC;
      const uint32_t e = n3 * static_cast<uint32_t>(k2);  // < L2*L3
      float2 v = data[Lay::idx(k2, c)];
      v = cmul(v, cmul(wc, cmul(hi[e >> kP2LoBits], lo[e & (kLo - 1)])));
      BRP_ST(&base[static_cast<size_t>(k2) * a.L3 + c], v);
    }
    if (a.partials != nullptr && rem == 0) reduce_delta<NT>(a, b, red);
    __syncthreads();  // LDS tile free for the next iteration
    tile = next;
  }
}

// Register-staged pass 2 for L = R1 * 16 with R1 | 16 (L in 32..256), the
// two-stage radix (R1, 16) transform of 16 columns. The columns a thread loads
// (rows tj + TPC u) are exactly the inputs of its stage-1 butterflies, and the
// rows its stage-2 butterfly produces (k2 = tj + TPC q) are exactly the rows it
// stores, so the tile crosses LDS once (stage 1 -> stage 2) instead of four
// times, with two barriers per tile. The output twiddle
// W_M^{n3 (k1 + L1 k2)} = wc * W_{L2L3}^{n3 tj} * (W_{L2L3}^{n3 TPC})^q is
// evaluated exactly at q = 0 and q = 8 and stepped by one rotation in between.
#ifndef BRP_P2R_WAVES
#define BRP_P2R_WAVES 3  // minimum waves per SIMD the register budget must allow (build switch)
#endif
template <int L, bool REV = false>
__global__ void __launch_bounds__(kNcol * (L / 16)) __attribute__((amdgpu_waves_per_eu(BRP_P2R_WAVES, 8))) pass2r_kernel(Pass2Args a, uint32_t ntiles) {
  constexpr int R1 = L / 16;
  constexpr int TPC = R1;
  constexpr int NT = kNcol * TPC;
  constexpr int NB1 = 16 / R1;  // stage-1 butterflies per thread
  static_assert(R1 >= 2 && 16 % R1 == 0, "L = R1 * 16 with R1 | 16");
  constexpr int kLo = 1 << kP2LoBits;
  __shared__ __attribute__((aligned(16))) float2 data[L * kNcol];
  __shared__ float2 wl[L];  // W_L^e
  __shared__ double red[NT / kWave + 1];
  const float2* lo = a.tb.p2lo;  // three exact lookups per tile: served by L1/L2
  const float2* hi = a.tb.p2hi;

  const uint32_t nblk3 = a.L3 / kNcol;
  const uint32_t per_b = a.L1 * nblk3;
  const size_t M = static_cast<size_t>(a.L1) * a.L2L3;
  const int c = threadIdx.x % kNcol;
  const int tj = threadIdx.x / kNcol;
  // wave-uniform tile origin, kept in SGPRs (the runtime divisions are VALU
  // sequences; readfirstlane lets every load/store use an SGPR base + 32-bit offset)
  auto tile_base = [&](uint32_t tl) -> const float2* {
    const uint32_t b = tl / per_b, rem = tl % per_b;
    const size_t off = static_cast<size_t>(b) * M + static_cast<size_t>(rem / nblk3) * a.L2L3 + (rem % nblk3) * kNcol;
    const uint32_t lo32 = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(off));
    const uint32_t hi32 = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(off >> 32));
    return a.buf + ((static_cast<size_t>(hi32) << 32) | lo32);
  };
  auto col = [](int r, int cc) { return r * kNcol + cc; };
  // per-lane byte offset of (row tj, column c) from a tile origin; row u*TPC
  // of the tile is a uniform (SGPR) base: one VGPR addresses all 16 accesses
  const uint32_t lane_off = (static_cast<uint32_t>(tj) * a.L3 + c) * sizeof(float2);
  const size_t row_step = static_cast<size_t>(TPC) * a.L3;
  auto at = [&](const float2* origin, int u) -> const float2* {
    return reinterpret_cast<const float2*>(reinterpret_cast<const char*>(origin + u * row_step) + lane_off);
  };

  float2 pre[16];
  uint32_t tile = blockIdx.x;
  if (tile < ntiles) {
    const float2* src = tile_base(tile);
#pragma unroll
    for (int u = 0; u < 16; ++u) pre[u] = BRP_LD(at(src, u));
  }
  {
    for (int e = threadIdx.x; e < L; e += NT) wl[e] = BRP_LD(&a.tb.st2[e + (e >> 4)]);
  }
  __syncthreads();
  while (tile < ntiles) {
    const uint32_t b = __builtin_amdgcn_readfirstlane(tile / per_b);
    const uint32_t rem = __builtin_amdgcn_readfirstlane(tile % per_b);
    const uint32_t k1 = __builtin_amdgcn_readfirstlane(rem / nblk3);
    const uint32_t n3 = (rem % nblk3) * kNcol + c;
    float2* base = const_cast<float2*>(tile_base(tile));
    const float2 wc = BRP_LD(&a.tb.p2col[k1 * a.L3 + n3]);
    // stage 1 (radix R1, no twiddles) on the loaded rows: butterfly
    // j = tj + R1 v holds rows j + 16 q = tj + TPC (v + NB1 q)
#pragma unroll
    for (int v = 0; v < NB1; ++v) {
      float2 x[R1];
#pragma unroll
      for (int q = 0; q < R1; ++q) x[q] = pre[v + NB1 * q];
      Dft<R1>::run(x);
      const int j = tj + R1 * v;
#pragma unroll
      for (int q = 0; q < R1; ++q) data[col(R1 * j + q, c)] = x[q];
    }
    const uint32_t next = tile + gridDim.x;
    if (next < ntiles) {  // in flight during the exchange, stage 2 and the stores
      const float2* src = tile_base(next);
#pragma unroll
      for (int u = 0; u < 16; ++u) pre[u] = BRP_LD(at(src, u));
    }
    __syncthreads();
    // stage 2 (radix 16, Ns = R1): butterfly tj reads rows tj + R1 q, twiddle W_L^{tj q}
    float2 y[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) y[q] = data[col(tj + R1 * q, c)];
    __syncthreads();  // LDS tile free for the next tile's stage 1
#pragma unroll
    for (int q = 1; q < 16; ++q) y[q] = cmul(y[q], wl[(tj * q) % L]);
    Dft<16>::run(y);
    if constexpr (REV) {
      // transposed inverse transform: outputs m2 = tj + TPC q with
      // W_{L1 L2}^{k1 m2} (p1 table, [m2][k1]), exact at q = 0 and 8 and
      // stepped by W_{L1 L2}^{k1 TPC} in between (as the forward twiddles)
      const float2* p1c = a.tb.p1 + k1;
      const float2 step = BRP_LD(&p1c[static_cast<uint32_t>(TPC) * a.L1]);
      float2 t0 = BRP_LD(&p1c[static_cast<uint32_t>(tj) * a.L1]);
      float2 t8 = BRP_LD(&p1c[static_cast<uint32_t>(tj + 8 * TPC) * a.L1]);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        BRP_ST(const_cast<float2*>(at(base, q)), cmul(y[q], t0));
        BRP_ST(const_cast<float2*>(at(base, q + 8)), cmul(y[q + 8], t8));
        t0 = cmul(t0, step);
        t8 = cmul(t8, step);
      }
      tile = next;
      continue;
    }
    // outputs k2 = tj + TPC q
    auto wexact = [&](uint32_t e) { return cmul(BRP_LD(&hi[e >> kP2LoBits]), BRP_LD(&lo[e & (kLo - 1)])); };
    const float2 step = wexact(n3 * static_cast<uint32_t>(TPC));
    float2 t0 = cmul(wc, wexact(n3 * static_cast<uint32_t>(tj)));
    float2 t8 = cmul(wc, wexact(n3 * static_cast<uint32_t>(tj + 8 * TPC)));
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      BRP_ST(const_cast<float2*>(at(base, q)), cmul(y[q], t0));
      BRP_ST(const_cast<float2*>(at(base, q + 8)), cmul(y[q + 8], t8));
      t0 = cmul(t0, step);
      t8 = cmul(t8, step);
    }
    if (a.partials != nullptr && rem == 0) reduce_delta<NT>(a, b, red);
    tile = next;
  }
}

// Composite radix R = A * B in registers (Cooley-Tukey, n = B n1 + n2,
// k = k1 + A k2), twiddles W_R^e from tw(e); radices with a Dft<> run it.
template <int R>
struct RadixKind {
  static constexpr bool kDirect = R == 2 || R == 3 || R == 4 || R == 5 || R == 7 || R == 8 || R == 16;
};
template <int R>
struct RadixSplit;  // R = A * B with A a direct radix
template <> struct RadixSplit<6> { static constexpr int A = 2, B = 3; };
template <> struct RadixSplit<9> { static constexpr int A = 3, B = 3; };
template <> struct RadixSplit<10> { static constexpr int A = 2, B = 5; };
template <> struct RadixSplit<12> { static constexpr int A = 3, B = 4; };
template <> struct RadixSplit<14> { static constexpr int A = 2, B = 7; };
template <> struct RadixSplit<15> { static constexpr int A = 3, B = 5; };
template <> struct RadixSplit<18> { static constexpr int A = 2, B = 9; };
template <> struct RadixSplit<20> { static constexpr int A = 4, B = 5; };
template <> struct RadixSplit<24> { static constexpr int A = 3, B = 8; };
template <> struct RadixSplit<28> { static constexpr int A = 4, B = 7; };
template <> struct RadixSplit<32> { static constexpr int A = 2, B = 16; };

template <int R, class TW>
__device__ __forceinline__ void dft_any(float2* v, TW tw) {
  if constexpr (RadixKind<R>::kDirect) {
    Dft<R>::run(v);
  } else {
    constexpr int A = RadixSplit<R>::A, B = RadixSplit<R>::B;
    float2 y[A][B];
#pragma unroll
    for (int n2 = 0; n2 < B; ++n2) {
      float2 t[A];
#pragma unroll
      for (int n1 = 0; n1 < A; ++n1) t[n1] = v[B * n1 + n2];
      Dft<A>::run(t);
#pragma unroll
      for (int k1 = 0; k1 < A; ++k1) y[k1][n2] = (k1 * n2 == 0) ? t[k1] : cmul(t[k1], tw(k1 * n2));
    }
    // W_B^e = W_R^{A e}
    auto twb = [&](int e) { return tw(A * e); };
#pragma unroll
    for (int k1 = 0; k1 < A; ++k1) {
      float2 t[B];
#pragma unroll
      for (int n2 = 0; n2 < B; ++n2) t[n2] = y[k1][n2];
      dft_any<B>(t, twb);
#pragma unroll
      for (int k2 = 0; k2 < B; ++k2) v[k1 + A * k2] = t[k2];
    }
  }
}

// Chirp factors w_n = W_{2 Mb}^{n^2 mod 2 Mb} along n_q = n0 + q D: exact at
// q = 0 and every 8 steps, in between w_{q+1} = w_q * r_q with
// r_q = W^{2 n_q D + D^2} and r_{q+1} = r_q * W^{2 D^2} (two complex products
// per element instead of a 64-bit reduction and two scattered table loads:
// n^2 mod 2 Mb lands anywhere in the table). 7 steps add a few ulp of phase.
struct ChirpWalk {
  const TwiddleTable& t;
  uint64_t n0, D;
  float2 w, r, c2;
  __device__ __forceinline__ ChirpWalk(const TwiddleTable& tt, uint64_t n0_, uint64_t D_) : t(tt), n0(n0_), D(D_) {
    c2 = tw_lookup(t, 2 * D * D);
  }
  // w_{n_q}; call with q = 0, 1, 2, ... in order
  __device__ __forceinline__ float2 next(int q) {
    if (q % 8 == 0) {
      const uint64_t n = n0 + static_cast<uint64_t>(q) * D;
      w = tw_lookup(t, n * n);
      r = tw_lookup(t, 2 * n * D + D * D);
    } else {
      w = cmul(w, r);
      r = cmul(r, c2);
    }
    return w;
  }
};
// stand-in for the modes without a reverse chirp: the table is unset there
// (period 0, no entries), so no lookup may be emitted at all
struct NoChirpWalk {
  __device__ __forceinline__ NoChirpWalk(const TwiddleTable&, uint64_t, uint64_t) {}
  __device__ __forceinline__ float2 next(int) { return make_float2(1.0f, 0.0f); }
};

// Register-staged pass 2 for L = 16 * R1 with R1 not a divisor of 16 (96, 144,
// 160, 192, 240, 288, 320: the chirp-z plans' lengths), two Stockham stages in
// the other order than pass2r_kernel: radix 16 first (butterfly tj of a column
// reads rows tj + R1 q, exactly the rows the thread loaded), then radix R1
// (Ns = 16, butterflies j < 16 read rows j + 16 q and produce the natural-order
// rows k2 = j + 16 q they store). The tile crosses LDS once; the generic
// LDS-staged kernel crossed it once per stage (measured 22.3 us per million
// elements at L2 = 288 against 5.4 for pass2r, profiles/kernel_stats_r4.txt).
template <int L, bool REV = false>
#ifndef BRP_P2G_WAVES
#define BRP_P2G_WAVES 2  // minimum waves per SIMD the register budget must allow (build switch)
#endif
__global__ void __launch_bounds__(kNcol * (L / 16)) __attribute__((amdgpu_waves_per_eu(BRP_P2G_WAVES, 8))) pass2g_kernel(Pass2Args a, uint32_t ntiles) {
  constexpr int R1 = L / 16;
  constexpr int TPC = R1;
  constexpr int NT = kNcol * TPC;
  constexpr int NB2 = (16 + TPC - 1) / TPC;  // stage-2 butterflies per thread (16 per column)
  static_assert(L % 16 == 0 && 16 % R1 != 0, "L = 16 R1, R1 not a divisor of 16 (pass2r_kernel)");
  constexpr int kLo = 1 << kP2LoBits;
  __shared__ __attribute__((aligned(16))) float2 data[L * kNcol];
  __shared__ float2 wl[L];  // W_L^e
  __shared__ double red[NT / kWave + 1];
  const float2* lo = a.tb.p2lo;
  const float2* hi = a.tb.p2hi;

  const uint32_t nblk3 = a.L3 / kNcol;
  const uint32_t per_b = a.L1 * nblk3;
  const size_t M = static_cast<size_t>(a.L1) * a.L2L3;
  const int c = threadIdx.x % kNcol;
  const int tj = threadIdx.x / kNcol;
  auto tile_base = [&](uint32_t tl) -> const float2* {
    const uint32_t b = tl / per_b, rem = tl % per_b;
    const size_t off = static_cast<size_t>(b) * M + static_cast<size_t>(rem / nblk3) * a.L2L3 + (rem % nblk3) * kNcol;
    const uint32_t lo32 = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(off));
    const uint32_t hi32 = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(off >> 32));
    return a.buf + ((static_cast<size_t>(hi32) << 32) | lo32);
  };
  auto col = [](int r, int cc) { return r * kNcol + cc; };
  // loads: rows tj + R1 q = (lane offset of row tj) + q * (uniform R1 rows);
  // stores: rows j + 16 q = (lane offset of row j) + q * (uniform 16 rows):
  // one VGPR per access pattern, the row steps stay scalar
  const uint32_t ld_off = (static_cast<uint32_t>(tj) * a.L3 + c) * sizeof(float2);
  const size_t ld_step = static_cast<size_t>(R1) * a.L3;
  const size_t st_step = static_cast<size_t>(16) * a.L3;
  auto ld_at = [&](const float2* origin, int q) -> const float2* {
    return reinterpret_cast<const float2*>(reinterpret_cast<const char*>(origin + q * ld_step) + ld_off);
  };
  // W_{R1}^e = W_L^{16 e}
  auto tw1 = [&](int e) { return wl[(16 * e) % L]; };

  float2 pre[16];
  uint32_t tile = blockIdx.x;
  if (tile < ntiles) {
    const float2* src = tile_base(tile);
#pragma unroll
    for (int q = 0; q < 16; ++q) pre[q] = BRP_LD(ld_at(src, q));
  }
  for (int e = threadIdx.x; e < L; e += NT) wl[e] = BRP_LD(&a.tb.st2[e + (e >> 4)]);
  __syncthreads();
  while (tile < ntiles) {
    const uint32_t b = __builtin_amdgcn_readfirstlane(tile / per_b);
    const uint32_t rem = __builtin_amdgcn_readfirstlane(tile % per_b);
    const uint32_t k1 = __builtin_amdgcn_readfirstlane(rem / nblk3);
    const uint32_t n3 = (rem % nblk3) * kNcol + c;
    float2* base = const_cast<float2*>(tile_base(tile));
    const float2 wc = BRP_LD(&a.tb.p2col[k1 * a.L3 + n3]);
    // stage 1 (radix 16, Ns = 1): butterfly tj, outputs rows 16 tj + q
    Dft<16>::run(pre);
#pragma unroll
    for (int q = 0; q < 16; ++q) data[col(16 * tj + q, c)] = pre[q];
    const uint32_t next = tile + gridDim.x;
    if (next < ntiles) {  // in flight during the exchange, stage 2 and the stores
      const float2* src = tile_base(next);
#pragma unroll
      for (int q = 0; q < 16; ++q) pre[q] = BRP_LD(ld_at(src, q));
    }
    __syncthreads();
    // stage 2 (radix R1, Ns = 16): butterfly j reads rows j + 16 q, twiddle W_L^{j q}
    float2 y[NB2][R1];
#pragma unroll
    for (int v = 0; v < NB2; ++v) {
      const int j = tj + TPC * v;
      if (j < 16) {
#pragma unroll
        for (int q = 0; q < R1; ++q) y[v][q] = data[col(j + 16 * q, c)];
#pragma unroll
        for (int q = 1; q < R1; ++q) y[v][q] = cmul(y[v][q], wl[(j * q) % L]);
        dft_any<R1>(y[v], tw1);
      }
    }
    __syncthreads();  // LDS tile free for the next tile's stage 1
    if constexpr (REV) {
      // transposed inverse transform: outputs m2 = j + 16 q with
      // W_{L1 L2}^{k1 m2} (p1 table, [m2][k1]), exact every 8 rows and
      // stepped by W_{L1 L2}^{16 k1} in between (as the forward twiddles)
      const float2* p1c = a.tb.p1 + k1;
      const float2 step = BRP_LD(&p1c[16u * a.L1]);
#pragma unroll
      for (int v = 0; v < NB2; ++v) {
        const int j = tj + TPC * v;
        if (j < 16) {
          const uint32_t st_off = (static_cast<uint32_t>(j) * a.L3 + c) * sizeof(float2);
          float2 t = make_float2(1.f, 0.f);
#pragma unroll
          for (int q = 0; q < R1; ++q) {
            if (q % 8 == 0) t = BRP_LD(&p1c[static_cast<uint32_t>(j + 16 * q) * a.L1]);
            BRP_ST(reinterpret_cast<float2*>(reinterpret_cast<char*>(base + q * st_step) + st_off), cmul(y[v][q], t));
            t = cmul(t, step);
          }
        }
      }
      tile = next;
      continue;
    }
    // outputs k2 = j + 16 q with W_M^{n3 (k1 + L1 k2)} = wc * W_{L2L3}^{n3 k2},
    // exact every 8 rows and stepped by W_{L2L3}^{16 n3} in between
    auto wexact = [&](uint32_t e) { return cmul(BRP_LD(&hi[e >> kP2LoBits]), BRP_LD(&lo[e & (kLo - 1)])); };
    const float2 step = wexact(n3 * 16u);
#pragma unroll
    for (int v = 0; v < NB2; ++v) {
      const int j = tj + TPC * v;
      if (j < 16) {
        const uint32_t st_off = (static_cast<uint32_t>(j) * a.L3 + c) * sizeof(float2);
        float2 t = make_float2(1.f, 0.f);
#pragma unroll
        for (int q = 0; q < R1; ++q) {
          if (q % 8 == 0) t = cmul(wc, wexact(n3 * static_cast<uint32_t>(j + 16 * q)));
          BRP_ST(reinterpret_cast<float2*>(reinterpret_cast<char*>(base + q * st_step) + st_off), cmul(y[v][q], t));
          t = cmul(t, step);
        }
      }
    }
    if (a.partials != nullptr && rem == 0) reduce_delta<NT>(a, b, red);
    tile = next;
  }
}

// Register-staged pass 1, L1 = 16 R1, for the chirp-z transforms (complex
// input: P1_COMPLEX / P1_COMPLEX_CONJ; the chirp-multiplied resampled series:
// P1_CHIRP2 / P1_CHIRP1 / P1_CHIRP1_PAIR, zero from Mb on) and for the
// resampling gather of the lengths without a pruned kernel (P1_RESAMPLE: e.g.
// L1 = 224 for -P 3.5, N = 7 * 2^21): the pass2g_kernel order -- radix 16 on
// the rows a thread loads (tj + R1 q), one LDS crossing, radix R1 producing
// the natural-order rows k1 = j + 16 q it stores with the output twiddle
// W_{L1 L2}^{n2 k1}. The LDS-staged pass1_kernel crosses LDS once per stage
// and bounds the chirp-z transforms (profiles/README.md, round 4).
template <int L, int MODE>
#ifndef BRP_P1G_WAVES
#define BRP_P1G_WAVES 2  // minimum waves per SIMD the register budget must allow (build switch)
#endif
__global__ void __launch_bounds__(kNcol * (L / 16)) __attribute__((amdgpu_waves_per_eu(BRP_P1G_WAVES, 8))) pass1g_kernel(Pass1Args a) {
  constexpr int R1 = L / 16;
  constexpr int TPC = R1;
  constexpr int NB2 = (16 + TPC - 1) / TPC;  // stage-2 butterflies per thread (16 per column)
  constexpr bool kChirp = MODE == P1_CHIRP2 || MODE == P1_CHIRP1 || MODE == P1_CHIRP1_PAIR;
  static_assert(kChirp || MODE == P1_COMPLEX || MODE == P1_COMPLEX_CONJ || MODE == P1_RESAMPLE || MODE == P1_REV_CHIRP,
                "pass1g modes");
  constexpr int NT = kNcol * TPC;
  __shared__ __attribute__((aligned(16))) float2 data[L * kNcol];
  __shared__ float2 wl[L];  // W_L^e
  __shared__ float lut_s[kLutSize], lut_c[kLutSize];
  __shared__ double red[NT / kWave + 1];

  const int b = blockIdx.y;
  const uint32_t nblk3 = a.L3 / kNcol;
  const uint32_t n2 = blockIdx.x / nblk3;
  const uint32_t col_base = n2 * a.L3 + (blockIdx.x % nblk3) * kNcol;
  const size_t M = static_cast<size_t>(L) * a.L2L3;
  const int c = threadIdx.x % kNcol;
  const int tj = threadIdx.x / kNcol;
  auto col = [](int r, int cc) { return r * kNcol + cc; };
  auto tw1 = [&](int e) { return wl[(16 * e) % L]; };  // W_{R1}^e = W_L^{16 e}
  if (a.reset != nullptr && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) BRP_ST(a.reset, 0u);

  float2 x[16];
  double sum = 0.0, sum_b = 0.0;  // sum_b: the second template of a pair (P1_CHIRP1_PAIR)
  if constexpr (MODE == P1_RESAMPLE) {
    // nearest-neighbour resampling of rows tj + R1 q (pass1_kernel's
    // arithmetic): all 32 indices first (LUT sine, VALU), then all loads in
    // flight together, then centring and the partial sum
    for (int i = threadIdx.x; i < kLutSize; i += NT) {
      lut_s[i] = kSinLut[i];
      lut_c[i] = kCosLut[i];
    }
    __syncthreads();
    const bool fast = a.n_unpadded <= (1u << 23);
    const TemplateDev td = BRP_LD(&a.tmpl[b]);
    const float* series = a.series + static_cast<size_t>(td.wu) * a.n_unpadded;
    const int last = static_cast<int>(a.n_unpadded) - 1;
    int idx[32];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const uint32_t m0 = 2 * (static_cast<uint32_t>(tj + R1 * q) * a.L2L3 + col_base + c);
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
    for (int e = 0; e < 32; ++e) raw[e] = BRP_LD(&series[idx[e] < 0 ? 0 : idx[e]]);
    float fsum = 0.0f;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const float x0 = idx[2 * q] < 0 ? 0.0f : raw[2 * q] - td.mu0;
      const float x1 = idx[2 * q + 1] < 0 ? 0.0f : raw[2 * q + 1] - td.mu0;
      fsum += x0 + x1;
      x[q] = make_float2(x0, x1);
    }
    sum = static_cast<double>(fsum);
  } else if constexpr (!kChirp) {
    // rows tj + R1 q: uniform row step R1 L2L3, one lane offset
    const float2* src = a.cplx_in + static_cast<size_t>(b) * M + col_base + c + static_cast<size_t>(tj) * a.L2L3;
    const size_t ld_step = static_cast<size_t>(R1) * a.L2L3;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const float2 v = BRP_LD(&src[q * ld_step]);
      x[q] = MODE == P1_COMPLEX_CONJ ? conjf2(v) : v;
    }
  } else {
    // the resampled series times the chirp W_{2Mb}^{n^2}, zero from Mb on
    // (same arithmetic as pass1_kernel's chirp modes)
    for (int i = threadIdx.x; i < kLutSize; i += NT) {
      lut_s[i] = kSinLut[i];
      lut_c[i] = kCosLut[i];
    }
    __syncthreads();
    constexpr bool kPair = MODE == P1_CHIRP1_PAIR;
    const bool fast = a.n_unpadded <= (1u << 23);
    const int ta = kPair ? 2 * b : b;
    const bool has_b = kPair && static_cast<uint32_t>(ta + 1) < a.n_tmpl;
    const TemplateDev td = BRP_LD(&a.tmpl[ta]);
    TemplateDev tdb = td;
    if (has_b) tdb = BRP_LD(&a.tmpl[ta + 1]);
    const float* series = a.series + static_cast<size_t>(td.wu) * a.n_unpadded;
    const float* series_b = a.series + static_cast<size_t>(tdb.wu) * a.n_unpadded;
    const int last = static_cast<int>(a.n_unpadded) - 1;
    auto sample_of = [&](const TemplateDev& t, const float* ser, uint32_t m) -> float {
      if (m >= t.n_steps) return 0.0f;
      const float dt = resamp_del_t(m, t.p, lut_s, lut_c);
      const int i = min(max(fast ? resamp_nearest_f(m, dt) : resamp_nearest(m, dt), 0), last);
      return BRP_LD(&ser[i]) - t.mu0;
    };
    (void)sample_of;
    // three phases as the resampling gather: the nearest indices of all 16
    // rows (two samples each: the pair (2n, 2n + 1), or templates a and b),
    // all loads in flight together, then centring, chirp and the sums
    const uint32_t n0 = static_cast<uint32_t>(tj) * a.L2L3 + col_base + c;
    const uint32_t D = static_cast<uint32_t>(R1) * a.L2L3;
    // rows q >= qw of the whole wave lie in the zero padding (n >= Mb, about
    // half the rows): their gathers and chirp factors are skipped uniformly
    const uint32_t qw = wave_max_u32<5>(n0 < a.Mb ? min(16u, (a.Mb - n0 + D - 1) / D) : 0u);
    int idx[32];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const uint32_t n = n0 + q * D;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const TemplateDev& t = (MODE == P1_CHIRP2 || h == 0) ? td : tdb;
        const uint32_t m = MODE == P1_CHIRP2 ? 2 * n + h : n;
        int i = -1;
        if (n < a.Mb && m < t.n_steps && (MODE == P1_CHIRP2 || h == 0 || has_b)) {
          const float dt = resamp_del_t(m, t.p, lut_s, lut_c);
          i = min(max(fast ? resamp_nearest_f(m, dt) : resamp_nearest(m, dt), 0), last);
        }
        idx[2 * q + h] = i;
      }
    }
    // loads in two halves of 8 rows; the second only when a row of the wave
    // needs it (uniform branch: a per-row guard spilled the arrays)
    float raw[32];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const float* ser = (MODE == P1_CHIRP2 || e % 2 == 0) ? series : series_b;
      raw[e] = BRP_LD(&ser[idx[e] < 0 ? 0 : idx[e]]);
    }
#pragma unroll
    for (int e = 16; e < 32; ++e) raw[e] = 0.0f;
    if (qw > 8) {
#pragma unroll
      for (int e = 16; e < 32; ++e) {
        const float* ser = (MODE == P1_CHIRP2 || e % 2 == 0) ? series : series_b;
        raw[e] = BRP_LD(&ser[idx[e] < 0 ? 0 : idx[e]]);
      }
    }
    float fsum = 0.0f, fsum_b = 0.0f;
    ChirpWalk cw(a.chirp, n0, D);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      float2 v = make_float2(0.0f, 0.0f);
      if (static_cast<uint32_t>(q) < qw) {
        const float2 w = cw.next(q);  // W_{2Mb}^{n^2 mod 2Mb}
        const float s0 = idx[2 * q] < 0 ? 0.0f : raw[2 * q] - td.mu0;
        const float s1 = idx[2 * q + 1] < 0 ? 0.0f : raw[2 * q + 1] - (MODE == P1_CHIRP2 ? td.mu0 : tdb.mu0);
        const float2 xs = make_float2(s0, s1);
        if (MODE == P1_CHIRP2) {
          fsum += xs.x + xs.y;
        } else {
          fsum += xs.x;
          fsum_b += xs.y;
        }
        if (n0 + q * D < a.Mb) v = cmul(xs, w);
      }
      x[q] = v;
    }
    sum = static_cast<double>(fsum);
    sum_b = static_cast<double>(fsum_b);
  }
  for (int e = threadIdx.x; e < L; e += NT) wl[e] = BRP_LD(&a.tb.st1[e + (e >> 4)]);
  // stage 1 (radix 16, Ns = 1): butterfly tj, outputs rows 16 tj + q
  Dft<16>::run(x);
#pragma unroll
  for (int q = 0; q < 16; ++q) data[col(16 * tj + q, c)] = x[q];
  __syncthreads();
  // stage 2 (radix R1, Ns = 16): butterfly j reads rows j + 16 q, twiddle W_L^{j q};
  // outputs k1 = j + 16 q with W_{L1 L2}^{n2 k1} (p1 table)
  float2* out = a.out + static_cast<size_t>(b) * M + col_base + c;
  const float2* two = a.tb.p1 + static_cast<size_t>(n2) * L;
#pragma unroll
  for (int v = 0; v < NB2; ++v) {
    const int j = tj + TPC * v;
    if (j < 16) {
      // P1_REV_CHIRP: chirp factors of the outputs n = (j + 16 q) L2L3 + col
      std::conditional_t<MODE == P1_REV_CHIRP, ChirpWalk, NoChirpWalk> cw(
          a.chirp, static_cast<uint64_t>(j) * a.L2L3 + col_base + c, 16ull * a.L2L3);
      float2 y[R1];
#pragma unroll
      for (int q = 0; q < R1; ++q) y[q] = data[col(j + 16 * q, c)];
#pragma unroll
      for (int q = 1; q < R1; ++q) y[q] = cmul(y[q], wl[(j * q) % L]);
      dft_any<R1>(y, tw1);
#pragma unroll
      for (int q = 0; q < R1; ++q) {
        const int k1 = j + 16 * q;
        if constexpr (MODE == P1_REV_CHIRP) {
          // natural-order n: conj(.) * w_n / L for n < Mb (the length-Mb DFT)
          const uint32_t n = static_cast<uint32_t>(k1) * a.L2L3 + col_base + c;
          const float2 w = cw.next(q);
          if (n < a.Mb) BRP_ST(&out[static_cast<size_t>(k1) * a.L2L3], cscale(cmul(conjf2(y[q]), w), a.scale));
        } else {
          BRP_ST(&out[static_cast<size_t>(k1) * a.L2L3], cmul(y[q], BRP_LD(&two[k1])));
        }
      }
    }
  }
  if constexpr (MODE == P1_CHIRP2 || MODE == P1_CHIRP1 || MODE == P1_RESAMPLE) {
    const double tot = block_sum<NT>(sum, red);
    if (threadIdx.x == 0) BRP_ST(&a.partials[static_cast<size_t>(b) * gridDim.x + blockIdx.x], tot);
  } else if constexpr (MODE == P1_CHIRP1_PAIR) {  // partial sums per template (2b, 2b + 1)
    const double tot = block_sum<NT>(sum, red);
    const double tot_b = block_sum<NT>(sum_b, red);
    if (threadIdx.x == 0) {
      BRP_ST(&a.partials[static_cast<size_t>(2 * b) * gridDim.x + blockIdx.x], tot);
      if (static_cast<uint32_t>(2 * b + 1) < a.n_tmpl)
        BRP_ST(&a.partials[static_cast<size_t>(2 * b + 1) * gridDim.x + blockIdx.x], tot_b);
    }
  }
}

// ------------------------------------------------------------------ pass 3
__device__ __forceinline__ size_t row_base(uint32_t c, uint32_t L1, uint32_t L2, uint32_t L3) {
  const uint32_t k1 = c % L1, k2 = c / L1;
  return (static_cast<size_t>(k1) * L2 + k2) * L3;
}

__device__ __forceinline__ float2 padding_spectrum(const TwiddleTable& tw, uint32_t n_s, uint32_t k) {
  return padding_spectrum_t(tw_lookup(tw, static_cast<uint64_t>(n_s) * k), tw_lookup32(tw, k),
                            tw_lookup(tw, static_cast<uint64_t>(n_s - 1) * k));
}

// Per-row constants: bin k = c + C k3 factors as W_2N^{x k} = W_2N^{x c} * W_{4 L3}^{x k3}
struct RowTw {
  float2 t1;  // W_2N^c
  float2 ta;  // W_2N^{n_s c}
};

__device__ __forceinline__ RowTw row_twiddles(const TwiddleTable& tw, uint32_t c, uint32_t n_s) {
  RowTw r;
  r.t1 = tw_lookup32(tw, c);
  r.ta = tw_lookup(tw, static_cast<uint64_t>(n_s) * c);
  return r;
}

// Output of one untangled bin: X_k (+ delta * S_k) -> |X_k|^2 / N (fp32 or
// fp16 spectrum), or the complex bin. S_k = -(sin(pi n_s k/N) / sin(pi k/N))
// e^{-i pi (n_s-1) k/N} from ta = W_2N^{n_s k}, tk = W_2N^k.
template <int MODE>
struct P3Emit {
  static constexpr bool kPower = (MODE == P3_POWER || MODE == P3_POWER16);
  const Pass3Args& a;
  float dS;
  bool correct;
  int b;
  __device__ __forceinline__ float power(uint32_t k, float2 x, float2 tk, float2 ta) const {
    if (k == 0) return 0.0f;
    if (correct) {
      const float ratio = ta.y * __builtin_amdgcn_rcpf(tk.y);  // v_rcp_f32 (1 ulp)
      const float2 tc = cmulc(ta, tk);                         // W_2N^{(n_s-1) k}
      x = cfma(-dS * ratio, tc, x);
    }
    const f2v xv = vec(x);
    const f2v sq = xv * xv;
    return (sq.x + sq.y) * a.norm;
  }
  // stores bin k's power; returns the value the spectrum holds (fp16-rounded in P3_POWER16)
  __device__ __forceinline__ float store(uint32_t k, float p) const {
    const size_t o = BRP_INJECT_AT(static_cast<size_t>(b) * a.ps_stride + k,
                                   static_cast<size_t>(gridDim.y) * a.ps_stride + 16, kInjPass3);
    // fp16 spectrum (config 5) saturates at the largest finite half: a strong
    // line stays a (clamped) candidate instead of an inf in the sums
    if (MODE == P3_POWER16) {
      const _Float16 h = static_cast<_Float16>(fminf(p, 65504.0f));
      BRP_ST(&a.ps16[o], h);
      return static_cast<float>(h);
    }
    BRP_ST(&a.ps[o], p);
    return p;
  }
  // the spectrum value written for bin k (0 for bins past the limit: the
  // harmonic sum never reads them, and the cell maxima count them as 0)
  __device__ __forceinline__ float operator()(uint32_t k, float2 x, float2 tk, float2 ta) const {
    if (k >= a.limit) return 0.0f;
    if (kPower) return store(k, power(k, x, tk, ta));
    BRP_ST(&a.spec[k], x);
    return 0.0f;
  }
  // Nyquist bin M: X_M = Re Z_0 - Im Z_0
  __device__ __forceinline__ float nyquist(float2 z0, uint32_t n_s) const {
    if (a.M >= a.limit) return 0.0f;
    float2 x = make_float2(z0.x - z0.y, 0.0f);
    if (kPower) {
      if (correct) {
        const float2 sp = padding_spectrum(a.tw, n_s, a.M);
        x = make_float2(x.x + dS * sp.x, x.y + dS * sp.y);
      }
      const float pm = (x.x * x.x + x.y * x.y) * a.norm;
      return store(a.M, pm);
    }
    BRP_ST(&a.spec[a.M], x);
    return 0.0f;
  }
};

// CELLS (power modes, a.cells set): the pruned harmonic sum's 8-bin bound
// cells of the rows' own bins fused into the untangle: the 8 rows c0 .. c0 + 7
// of a workgroup are the 8 consecutive bins of one aligned cell for every k3,
// held by 8 consecutive lanes (three shuffles), and no other workgroup writes
// that cell (residues below C/2). Their mirror bins M - k fall into two cells
// shared with the neighbouring workgroup: those cells (residues >= C/2) are
// left to hs_cells_kernel's mirror-half mode, which then reads half the
// spectrum. (A first form wrote the mirror cells too, with device-scope
// atomic max: pass 3 went from 41.9 to 74.0 us per template, round 6.)
template <int L, int ROWS, int MODE, bool CELLS = false>
__global__ void __launch_bounds__(2 * ROWS * tpc_for<L>()) pass3_kernel(Pass3Args a) {
  static_assert(!CELLS || ROWS == 8, "fused cells: one workgroup row group per 8-bin cell");
  constexpr int TPC = tpc_for<L>();
  constexpr int NSLOT = 2 * ROWS;
  constexpr int NT = NSLOT * TPC;
  constexpr int L4 = 4 * L;
  using Lay = BlockLayout<L, NSLOT, TPC, true>;
  // data | stage twiddles W_L | W_{4L} (= W_2N^{C i}) as lo[32] | hi[4L/32]
  constexpr int kT4 = 32 + L4 / 32;
  static_assert(L4 % 32 == 0, "two-level W_{4L} table");
  __shared__ __attribute__((aligned(16))) float2 smem[Lay::kLds + kTwPad<L> + kTwRowExtra<L> + kT4];
  float2* data = smem;
  float2* twl = smem + Lay::kLds;
  float2* t4 = twl + kTwPad<L> + kTwRowExtra<L>;
  // W_{4L}^j, j < 4L
  auto w4 = [&](uint32_t j) { return cmul(t4[32 + (j >> 5)], t4[j & 31u]); };

  const int b = blockIdx.y;
  const float2* buf = a.buf + static_cast<size_t>(b) * a.M;
  // neighbouring row blocks write neighbouring 32-B pieces of the same output
  // lines: keep them on one XCD so its L2 merges full lines
  const uint32_t c0 = xcd_remap(blockIdx.x, gridDim.x) * ROWS;

  // stage 1 (radix R0, Ns = 1) straight from global memory: butterfly
  // j = tj + TPC u reads elements j + (L/R0) q of its row (lanes walk j:
  // contiguous 8-B loads), transforms in registers and writes its Stockham
  // output rows R0 j + q to LDS; the remaining stages run LDS -> LDS
  constexpr int R0 = BlockFFT<L, NSLOT, TPC, true>::kFirstRadix;
  constexpr int kBf0 = L / R0;
  // Measured on MI355X (L = 256): 16-B row loads into LDS beat the 8-B loads
  // the register first stage needs (18.2 vs 18.9 us/template), so the
  // register path is kept for reference but disabled.
#ifdef BRP_P3_REG_STAGE1
  constexpr bool kRegStage1 = (kBf0 % TPC == 0);
#else
  constexpr bool kRegStage1 = false && (kBf0 % TPC == 0);
#endif
  // Every global load of the prologue is issued before the first LDS write:
  // row segments, stage twiddles, W_{4L} table. (A copy loop that stored each
  // twiddle before loading the next added 3 memory round trips after the rows
  // had arrived.)
  constexpr int kTwN = kTwPad<L> + kTwRowExtra<L>;
  constexpr int kTwIt = (kTwN + NT - 1) / NT;
  static_assert(kT4 <= NT, "one W_{4L} entry per thread");
  float2 twv[kTwIt];
  float2 t4v = make_float2(0.0f, 0.0f);
  auto load_tables = [&] {
#pragma unroll
    for (int i = 0; i < kTwIt; ++i) {
      const int e = static_cast<int>(threadIdx.x) + i * NT;
      twv[i] = e < kTwN ? BRP_LD(&a.tb.st3[e]) : make_float2(0.0f, 0.0f);
    }
    if (threadIdx.x < kT4) t4v = BRP_LD(&a.tb.p3[threadIdx.x]);
  };
  if constexpr (!kRegStage1) {
    int slot, tj;
    Lay::coords(threadIdx.x, slot, tj);
    const uint32_t cs = c0 + (slot % ROWS);
    const uint32_t row = (slot < ROWS) ? cs : (a.C - cs) % a.C;
    const float4* src = reinterpret_cast<const float4*>(buf + row_base(row < a.C ? row : 0, a.L1, a.L2, a.L3));
    constexpr int kRowIt = (L / 2) / TPC;
    static_assert((L / 2) % TPC == 0, "whole row-load iterations");
    float4 rv[kRowIt];
#pragma unroll
    for (int u = 0; u < kRowIt; ++u) rv[u] = BRP_LD(&src[tj + u * TPC]);
    load_tables();
#pragma unroll
    for (int u = 0; u < kRowIt; ++u) {
      const int r = tj + u * TPC;
      data[Lay::idx(2 * r, slot)] = make_float2(rv[u].x, rv[u].y);
      data[Lay::idx(2 * r + 1, slot)] = make_float2(rv[u].z, rv[u].w);
    }
  } else {
    int slot, tj;
    Lay::coords(threadIdx.x, slot, tj);
    const uint32_t cs = c0 + (slot % ROWS);
    const uint32_t row = (slot < ROWS) ? cs : (a.C - cs) % a.C;
    const float2* src = buf + row_base(row < a.C ? row : 0, a.L1, a.L2, a.L3);
    float2 v[kBf0 / TPC][R0];
#pragma unroll
    for (int u = 0; u < kBf0 / TPC; ++u)
#pragma unroll
      for (int q = 0; q < R0; ++q) v[u][q] = BRP_LD(&src[tj + u * TPC + q * kBf0]);
    load_tables();
#pragma unroll
    for (int u = 0; u < kBf0 / TPC; ++u) {
      Dft<R0>::run(v[u]);
      const int j = tj + u * TPC;
#pragma unroll
      for (int q = 0; q < R0; ++q) data[Lay::idx(R0 * j + q, slot)] = v[u][q];
    }
  }
#pragma unroll
  for (int i = 0; i < kTwIt; ++i) {
    const int e = static_cast<int>(threadIdx.x) + i * NT;
    if (e < kTwN) twl[e] = twv[i];
  }
  if (threadIdx.x < kT4) t4[threadIdx.x] = t4v;
  // mean-padding correction delta = (sum of (sample - mu0)) / n_steps (pass 2)
  double delta = 0.0;
  uint32_t n_s = 0;
  if (MODE == P3_POWER || MODE == P3_POWER16) {
    n_s = BRP_LD(&a.tmpl[b]).n_steps;
    delta = BRP_LD(&a.delta[b]);
  }
  // per-row twiddle constants of the untangle phase, fetched before the FFT so
  // their latency hides under it
  const int s = threadIdx.x % ROWS;
  const int t = threadIdx.x / ROWS;
  constexpr int kStreams = NT / ROWS;
  const uint32_t c = c0 + s;
  const uint32_t half = a.C / 2;
  const RowTw rt = row_twiddles(a.tw, c, n_s);
  __syncthreads();
  if constexpr (kRegStage1) BlockFFT<L, NSLOT, TPC, true>::run_rest(data, twl);
  else if constexpr (!kAblateP3Fft) BlockFFT<L, NSLOT, TPC, true>::run(data, twl);

  constexpr bool kPower = (MODE == P3_POWER || MODE == P3_POWER16);
  const bool correct = kPower && n_s > 0;
  P3Emit<MODE> emit{a, static_cast<float>(delta), correct, b};

  // untangle: thread -> (slot s, k3 stream), rows c <= C/2 own their bins;
  // bin M-k of the mirror row reuses the twiddles of bin k:
  //   W_2N^{M-k} = -i conj(W_2N^k),  W_2N^{n_s (M-k)} = (-i)^{n_s} conj(W_2N^{n_s k})
  // The thread's bins k3 = t + kStreams * it advance the twiddles by fixed
  // rotations: W_2N^k and W_2N^{n_s k} are stepped by one complex multiply per
  // bin (a few ulp over L / kStreams steps) instead of two table products.
  static_assert(L % kStreams == 0, "whole untangle iterations");
  const bool live = c <= half;  // rows beyond C/2 are the mirrors of others
  // cells of this template; the workgroup's own cells are its alone unless its
  // rows reach C/2 (that cell also holds mirror bins of the workgroup before)
  float* const cells = CELLS ? a.cells + static_cast<size_t>(b) * a.cells_stride : nullptr;
  const bool own_excl = c0 + ROWS <= half;  // the workgroup at C/2 leaves its cell to hs_cells_kernel
  auto group_max = [](float v) {
    v = fmaxf(v, __shfl_xor(v, 1, 8));
    v = fmaxf(v, __shfl_xor(v, 2, 8));
    return fmaxf(v, __shfl_xor(v, 4, 8));
  };
  if (CELLS || live) {
    float2 tk = cmul(rt.t1, w4(static_cast<uint32_t>(t)));  // W_2N^k for k3 = t
    const float2 tk_step = w4(static_cast<uint32_t>(kStreams));
    float2 ta = make_float2(0.f, 0.f), ta_step = make_float2(1.f, 0.f);
    // (-i)^{n_s}: W_2N^{n_s (M-k)} = (-i)^{n_s} conj(W_2N^{n_s k}) for the mirror bins
    const float2 rq = rot_mi(make_float2(1.f, 0.f), n_s);
    if (correct) {
      ta = cmul(rt.ta, w4((n_s * static_cast<uint32_t>(t)) % L4));
      ta_step = w4((n_s * static_cast<uint32_t>(kStreams)) % L4);
    }
#pragma unroll
    for (int it = 0; it < L / kStreams; ++it) {
      const int k3 = t + it * kStreams;
      if (it > 0) {
        tk = cmul(tk, tk_step);
        if (correct) ta = cmul(ta, ta_step);
      }
      const float2 zk = data[Lay::idx(k3, s)];
      const int k3m = (c == 0) ? (L - k3) % L : L - 1 - k3;
      const float2 zm = data[Lay::idx(k3m, c == 0 ? s : ROWS + s)];
      const uint32_t k = c + a.C * static_cast<uint32_t>(k3);
      const float2 w = cmul(tk, tk);          // W_N^k
      float v_own = 0.0f, v_mir = 0.0f, v_nyq = 0.0f;
      if (live) {
        v_own = emit(k, untangle_w(zk, zm, w), tk, ta);
        if (c != 0 && c != half) {
          const uint32_t kk = a.M - k;                 // = cm + C*(L-1-k3)
          const float2 tkm = make_float2(-tk.y, -tk.x);  // W_2N^{M-k} = -i conj(W_2N^k)
          const float2 tam = cmulc(rq, ta);
          v_mir = emit(kk, untangle_wm(zm, zk, w), tkm, tam);
        }
        if (c == 0 && k3 == 0) v_nyq = emit.nyquist(zk, n_s);
      }
      if constexpr (CELLS) {
        // every own cell is written, zeros included (bins past the limit):
        // the buffer is not cleared between batches
        const float m_own = group_max(v_own);
        const uint32_t idx = (c0 >> 3) + (a.C >> 3) * static_cast<uint32_t>(k3);
        if (s == 0 && own_excl && idx < a.n_cells) BRP_ST(&cells[idx], m_own);
      }
      (void)v_nyq;
    }
  }
}

template <int L, int ROWS>
__global__ void __launch_bounds__(ROWS * tpc_for<L>()) pass3_plain_kernel(Pass3PlainArgs a) {
  constexpr int TPC = tpc_for<L>();
  constexpr int NT = ROWS * TPC;
  using Lay = BlockLayout<L, ROWS, TPC, true>;
  __shared__ __attribute__((aligned(16))) float2 smem[Lay::kLds + kTwPad<L> + kTwRowExtra<L>];
  float2* data = smem;
  float2* twl = smem + Lay::kLds;
  const uint32_t c0 = blockIdx.x * ROWS;
  {
    int slot, tj;
    Lay::coords(threadIdx.x, slot, tj);
    const float2* src = a.buf + row_base(c0 + slot, a.L1, a.L2, a.L3);
    for (int r = tj; r < L; r += TPC) data[Lay::idx(r, slot)] = BRP_LD(&src[r]);
  }
  copy_row_twiddles<L>(twl, a.tb.st3);
  __syncthreads();
  BlockFFT<L, ROWS, TPC, true>::run(data, twl);
  // natural-order output z[c + C*k3] = conj(Z)*scale -> real samples 2n, 2n+1
  const int s = threadIdx.x % ROWS;
  const int t = threadIdx.x / ROWS;
  constexpr int kStreams = NT / ROWS;
  const uint32_t c = c0 + s;
  for (int k3 = t; k3 < L; k3 += kStreams) {
    const float2 z = data[Lay::idx(k3, s)];
    const size_t n = c + static_cast<size_t>(a.C) * k3;
    if (2 * n < a.n_out) BRP_ST(&a.real_out[2 * n], z.x * a.scale);
    if (2 * n + 1 < a.n_out) BRP_ST(&a.real_out[2 * n + 1], -z.y * a.scale);
  }
}

// Row pass of the chirp-z convolutions (bluestein_kernels.hpp): L3-point row
// FFTs of ROWS rows, natural-order complex output n = c + C k3 with the
// convolution's pointwise epilogue fused (multiply by H and conjugate, or the
// final chirp and 1/L), batched over blockIdx.y.
template <int L, int ROWS, int MODE>
__global__ void __launch_bounds__(ROWS * tpc_for<L>()) pass3_cplx_kernel(Pass3CplxArgs a) {
  constexpr int TPC = tpc_for<L>();
  constexpr int NT = ROWS * TPC;
  using Lay = BlockLayout<L, ROWS, TPC, true>;
  __shared__ __attribute__((aligned(16))) float2 smem[Lay::kLds + kTwPad<L> + kTwRowExtra<L>];
  float2* data = smem;
  float2* twl = smem + Lay::kLds;
  const int b = blockIdx.y;
  const uint32_t c0 = blockIdx.x * ROWS;
  const float2* buf = a.buf + static_cast<size_t>(b) * a.M;
  {
    int slot, tj;
    Lay::coords(threadIdx.x, slot, tj);
    const float2* src = buf + row_base(c0 + slot, a.L1, a.L2, a.L3);
    for (int r = tj; r < L; r += TPC) data[Lay::idx(r, slot)] = BRP_LD(&src[r]);
  }
  copy_row_twiddles<L>(twl, a.tb.st3);
  __syncthreads();
  BlockFFT<L, ROWS, TPC, true>::run(data, twl);
  const int s = threadIdx.x % ROWS;
  const int t = threadIdx.x / ROWS;
  constexpr int kStreams = NT / ROWS;
  const uint32_t c = c0 + s;
  float2* out = a.out + static_cast<size_t>(b) * a.out_stride;
  for (int k3 = t; k3 < L; k3 += kStreams) {
    const float2 z = data[Lay::idx(k3, s)];
    const uint32_t n = c + a.C * static_cast<uint32_t>(k3);
    if (MODE == C3_PLAIN) {
      BRP_ST(&out[n], z);
    } else if (MODE == C3_MULCONJ) {
      BRP_ST(&out[n], conjf2(cmul(z, BRP_LD(&a.h[n]))));
    } else if (n < a.n_out) {
      const float2 w = tw_lookup(a.chirp, static_cast<uint64_t>(n) * n);
      BRP_ST(&out[n], cscale(cmul(conjf2(z), w), a.scale));
    }
  }
}

// Middle of the transposed chirp-z convolution (Pass3MidArgs): ROWS
// consecutive rows of the row layout (row r = k1 L2 + k2 at r L3), forward
// row FFT, times H (same layout) and conj, second row FFT (the first pass of
// the transposed inverse transform), twiddle W_M^{m3 (k1 + L1 k2)}, stored
// back in place. Rows are contiguous in memory: whole-line loads and stores,
// where the natural-order epilogue of pass3_cplx_kernel wrote 64-B pieces.
template <int L, int ROWS>
__global__ void __launch_bounds__(ROWS * tpc_for<L>()) pass3_mid_kernel(Pass3MidArgs a) {
  constexpr int TPC = tpc_for<L>();
  constexpr int NT = ROWS * TPC;
  using Lay = BlockLayout<L, ROWS, TPC, true>;
  constexpr int kLo = 1 << kP2LoBits;
  __shared__ __attribute__((aligned(16))) float2 smem[Lay::kLds + kTwPad<L> + kTwRowExtra<L>];
  float2* data = smem;
  float2* twl = smem + Lay::kLds;
  const uint32_t M = a.L1 * a.L2 * a.L3;
  const uint32_t r0 = blockIdx.x * ROWS;
  float2* buf = a.buf + static_cast<size_t>(blockIdx.y) * M;
  int slot, tj;
  Lay::coords(threadIdx.x, slot, tj);
  const uint32_t row = r0 + slot;
  const size_t rbase = static_cast<size_t>(row) * L;
  constexpr int kPer = L / TPC;
  static_assert(L % TPC == 0, "whole row iterations");
  {
    float2 v[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u) v[u] = BRP_LD(&buf[rbase + tj + u * TPC]);
    copy_row_twiddles<L>(twl, a.tb.st3);
#pragma unroll
    for (int u = 0; u < kPer; ++u) data[Lay::idx(tj + u * TPC, slot)] = v[u];
  }
  __syncthreads();
  BlockFFT<L, ROWS, TPC, true>::run(data, twl);  // n3 -> k3 (natural order)
  {
    float2 h[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u) h[u] = BRP_LD(&a.hp[rbase + tj + u * TPC]);
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int e = Lay::idx(tj + u * TPC, slot);
      data[e] = conjf2(cmul(data[e], h[u]));
    }
  }
  __syncthreads();
  BlockFFT<L, ROWS, TPC, true>::run(data, twl);  // k3 -> m3
  // W_M^{m3 (k1 + L1 k2)} = W_M^{m3 k1} (p2col, contiguous in m3) *
  // W_{L2 L3}^{m3 k2}, the latter exact every 8 elements and stepped by
  // W_{L2 L3}^{TPC k2} in between (as pass 2's twiddles)
  const uint32_t k1 = row / a.L2, k2 = row % a.L2;
  const float2* wc = a.tb.p2col + static_cast<size_t>(k1) * L;
  auto wexact = [&](uint32_t e) { return cmul(BRP_LD(&a.tb.p2hi[e >> kP2LoBits]), BRP_LD(&a.tb.p2lo[e & (kLo - 1)])); };
  const float2 step = wexact(static_cast<uint32_t>(TPC) * k2);
  float2 t = make_float2(1.f, 0.f);
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const uint32_t m3 = tj + u * TPC;
    if (u % 8 == 0) t = wexact(m3 * k2);
    BRP_ST(&buf[rbase + m3], cmul(data[Lay::idx(m3, slot)], cmul(BRP_LD(&wc[m3]), t)));
    t = cmul(t, step);
  }
}

}  // namespace

// ------------------------------------------------------------ dispatch glue
// Compiled lengths (any 16 * 2^a 3^b 5^c 7^d with a radix list in fft_block.hpp
// can be added): N/2 = L1 * L2 * L3 must factor over these sets.
#define BRP_P12_LENGTHS(X) \
  X(16) X(32) X(48) X(64) X(80) X(96) X(112) X(128) X(144) X(160) X(192) X(224) X(240) X(256) X(288) X(320) X(384) \
      X(448) X(512)
#define BRP_P3_LENGTHS(X) X(64) X(96) X(128) X(160) X(192) X(256) X(320)
// register-staged pass 2 (pass2r_kernel: R1 | 16; pass2g_kernel: the others)
#define BRP_P2R_LENGTHS(X) X(32) X(64) X(128) X(256)
#define BRP_P2G_LENGTHS(X) X(48) X(80) X(96) X(112) X(144) X(160) X(192) X(224) X(240) X(288) X(320) X(384) X(448) X(512)
// register-staged pass 1 (pass1g_kernel) of every mode but the resampling gather
#define BRP_P1G_LENGTHS(X) \
  X(48) X(64) X(80) X(96) X(112) X(128) X(144) X(160) X(192) X(224) X(240) X(256) X(288) X(320) X(384) X(448) X(512)

bool pass12_length_supported(uint32_t L) {
  switch (L) {
#define X(n) case n:
    BRP_P12_LENGTHS(X)
#undef X
    return true;
    default: return false;
  }
}

bool pass3_length_supported(uint32_t L) {
  switch (L) {
#define X(n) case n:
    BRP_P3_LENGTHS(X)
#undef X
    return true;
    default: return false;
  }
}

hipError_t launch_pass1(const FFTPlan3& plan, Pass1Mode mode, const Pass1Args& a, int batch, hipStream_t s) {
  const dim3 grid(plan.wg1(), batch);
  // padding >= 3x: every template's rows n1 >= L1/3 are zero (n_steps <= n_unpadded)
  const bool pad3 = mode == P1_RESAMPLE && plan.L1 % 3 == 0 &&
                    2ull * (plan.L1 / 3) * a.L2L3 >= a.n_unpadded;
  if (pad3 && plan.L1 == 192) {
    BRP_LAUNCH((pass1_pruned3_kernel<4>), grid, dim3(kNcol * 16), 0, s, a);
    return launch_status();
  }
  if (pad3 && plan.L1 == 96) {
    BRP_LAUNCH((pass1_pruned3_kernel<2>), grid, dim3(kNcol * 16), 0, s, a);
    return launch_status();
  }
#ifndef BRP_P1G
#define BRP_P1G 1  // register-staged complex-input pass 1 (build switch)
#endif
  // register-staged pass 1 (one LDS crossing); a.lds_pass1: the LDS-staged
  // pass1_kernel for the resampling gather instead (A/B switch, BRP_P1_LDS=1)
  if (BRP_P1G && mode != P1_REAL && !(mode == P1_RESAMPLE && a.lds_pass1)) {
    // lengths R1 | 16 and the long ones: complex-input and chirp modes only
    // (the resampling gather keeps its kernels there: pruned3 / LDS-staged)
    if (mode != P1_RESAMPLE) {
      switch (plan.L1) {
#define X(n)                                                                                                 \
  case n: {                                                                                                  \
    const dim3 blk(kNcol * (n / 16));                                                                        \
    if (mode == P1_COMPLEX) BRP_LAUNCH((pass1g_kernel<n, P1_COMPLEX>), grid, blk, 0, s, a);          \
    else if (mode == P1_COMPLEX_CONJ) BRP_LAUNCH((pass1g_kernel<n, P1_COMPLEX_CONJ>), grid, blk, 0, s, a); \
    else if (mode == P1_CHIRP2) BRP_LAUNCH((pass1g_kernel<n, P1_CHIRP2>), grid, blk, 0, s, a);       \
    else if (mode == P1_CHIRP1) BRP_LAUNCH((pass1g_kernel<n, P1_CHIRP1>), grid, blk, 0, s, a);       \
    else if (mode == P1_REV_CHIRP) BRP_LAUNCH((pass1g_kernel<n, P1_REV_CHIRP>), grid, blk, 0, s, a); \
    else BRP_LAUNCH((pass1g_kernel<n, P1_CHIRP1_PAIR>), grid, blk, 0, s, a);                         \
    return launch_status();                                                                                \
  }
        X(48) X(64) X(80) X(128) X(256) X(384) X(512)
#undef X
        default: break;
      }
    }
    switch (plan.L1) {
#define X(n)                                                                                         \
  case n: {                                                                                          \
    const dim3 blk(kNcol * (n / 16));                                                                \
    if (mode == P1_RESAMPLE) BRP_LAUNCH((pass1g_kernel<n, P1_RESAMPLE>), grid, blk, 0, s, a); \
    else if (mode == P1_COMPLEX) BRP_LAUNCH((pass1g_kernel<n, P1_COMPLEX>), grid, blk, 0, s, a); \
    else if (mode == P1_REV_CHIRP) BRP_LAUNCH((pass1g_kernel<n, P1_REV_CHIRP>), grid, blk, 0, s, a); \
    else if (mode == P1_COMPLEX_CONJ) BRP_LAUNCH((pass1g_kernel<n, P1_COMPLEX_CONJ>), grid, blk, 0, s, a); \
    else if (mode == P1_CHIRP2) BRP_LAUNCH((pass1g_kernel<n, P1_CHIRP2>), grid, blk, 0, s, a);             \
    else if (mode == P1_CHIRP1) BRP_LAUNCH((pass1g_kernel<n, P1_CHIRP1>), grid, blk, 0, s, a);             \
    else BRP_LAUNCH((pass1g_kernel<n, P1_CHIRP1_PAIR>), grid, blk, 0, s, a);                               \
    return launch_status();                                                                        \
  }
      X(96) X(112) X(144) X(160) X(192) X(224) X(240) X(288) X(320) X(448)
#undef X
      default: break;
    }
  }
  switch (plan.L1) {
#define X(n)                                                                                          \
  case n: {                                                                                           \
    const dim3 block(kNcol * tpc_for<n>());                                                           \
    if (mode == P1_RESAMPLE) BRP_LAUNCH((pass1_kernel<n, P1_RESAMPLE>), grid, block, 0, s, a); \
    else if (mode == P1_REAL) BRP_LAUNCH((pass1_kernel<n, P1_REAL>), grid, block, 0, s, a);    \
    else if (mode == P1_COMPLEX) BRP_LAUNCH((pass1_kernel<n, P1_COMPLEX>), grid, block, 0, s, a); \
    else if (mode == P1_CHIRP2) BRP_LAUNCH((pass1_kernel<n, P1_CHIRP2>), grid, block, 0, s, a);   \
    else if (mode == P1_CHIRP1) BRP_LAUNCH((pass1_kernel<n, P1_CHIRP1>), grid, block, 0, s, a);   \
    else if (mode == P1_CHIRP1_PAIR) BRP_LAUNCH((pass1_kernel<n, P1_CHIRP1_PAIR>), grid, block, 0, s, a); \
    else BRP_LAUNCH((pass1_kernel<n, P1_COMPLEX_CONJ>), grid, block, 0, s, a);                 \
    break;                                                                                            \
  }
    BRP_P12_LENGTHS(X)
#undef X
    default: return hipErrorInvalidValue;
  }
  return launch_status();
}

hipError_t launch_pass2(const FFTPlan3& plan, const Pass2Args& a, int batch, hipStream_t s) {
  const uint32_t ntiles = plan.wg2() * static_cast<uint32_t>(batch);
  const dim3 grid(plan.persist_wgs ? std::min(ntiles, plan.persist_wgs) : ntiles);
  // register-staged pass 2 where compiled (one LDS crossing per tile), the
  // generic LDS-staged kernel for the other lengths
  switch (plan.L2) {
#define X(n)                                                                                       \
  case n:                                                                                          \
    if (a.rev) BRP_LAUNCH((pass2r_kernel<n, true>), grid, dim3(kNcol * (n / 16)), 0, s, a, ntiles); \
    else BRP_LAUNCH((pass2r_kernel<n>), grid, dim3(kNcol * (n / 16)), 0, s, a, ntiles);   \
    return launch_status();
    BRP_P2R_LENGTHS(X)
#undef X
    default: break;
  }
  // register-staged, radix 16 then R1 (L2 = 16 R1, R1 not a divisor of 16);
  // BRP_P2G=0 (build switch): the LDS-staged kernel
#ifndef BRP_P2G
#define BRP_P2G 1
#endif
  if (BRP_P2G || a.rev) {
    switch (plan.L2) {
#define X(n)                                                                                       \
  case n:                                                                                          \
    if (a.rev) BRP_LAUNCH((pass2g_kernel<n, true>), grid, dim3(kNcol * (n / 16)), 0, s, a, ntiles); \
    else BRP_LAUNCH((pass2g_kernel<n>), grid, dim3(kNcol * (n / 16)), 0, s, a, ntiles);   \
    return launch_status();
      BRP_P2G_LENGTHS(X)
#undef X
      default: break;
    }
  }
  if (a.rev) return hipErrorInvalidValue;  // no reverse form of the LDS-staged kernel
  switch (plan.L2) {
#define X(n)                                                                \
  case n:                                                                   \
    BRP_LAUNCH((pass2_kernel<n>), grid, dim3(kNcol * tpc_for<n>()), 0, s, a, ntiles); \
    break;
    BRP_P12_LENGTHS(X)
#undef X
    default: return hipErrorInvalidValue;
  }
  return launch_status();
}

constexpr int kRows3 = 8;
#ifndef BRP_P3_ROWS
#define BRP_P3_ROWS 8  // untangle pass: own rows per workgroup (build switch, profiles/README.md)
#endif
constexpr int kRowsP = BRP_P3_ROWS;

hipError_t launch_pass3(const FFTPlan3& plan, Pass3Mode mode, const Pass3Args& a, int batch, hipStream_t s) {
  if (plan.rows3 != kRows3) return hipErrorInvalidValue;
  // rows per workgroup of the untangle pass (own rows; as many mirror rows)
  const dim3 grid(((plan.L1 * plan.L2) / 2 + kRowsP) / kRowsP, batch);
  switch (plan.L3) {
#define X(n)                                                                                              \
  case n: {                                                                                               \
    const dim3 block(2 * kRowsP * tpc_for<n>());                                                          \
    if (mode == P3_POWER && a.ps16 && a.cells)                                                            \
      BRP_LAUNCH((pass3_kernel<n, kRowsP, P3_POWER16, true>), grid, block, 0, s, a);                      \
    else if (mode == P3_POWER && a.ps16)                                                                  \
      BRP_LAUNCH((pass3_kernel<n, kRowsP, P3_POWER16>), grid, block, 0, s, a);                            \
    else if (mode == P3_POWER && a.cells)                                                                 \
      BRP_LAUNCH((pass3_kernel<n, kRowsP, P3_POWER, true>), grid, block, 0, s, a);                        \
    else if (mode == P3_POWER) BRP_LAUNCH((pass3_kernel<n, kRowsP, P3_POWER>), grid, block, 0, s, a); \
    else BRP_LAUNCH((pass3_kernel<n, kRowsP, P3_COMPLEX>), grid, block, 0, s, a);                 \
    break;                                                                                                \
  }
    BRP_P3_LENGTHS(X)
#undef X
    default: return hipErrorInvalidValue;
  }
  return launch_status();
}

hipError_t launch_pass3_cplx(const FFTPlan3& plan, Pass3CplxMode mode, const Pass3CplxArgs& a, int batch,
                             hipStream_t s) {
  const dim3 grid(plan.wg3_plain(), batch);
  switch (plan.L3) {
#define X(n)                                                                                                       \
  case n: {                                                                                                        \
    const dim3 block(kRows3 * tpc_for<n>());                                                                       \
    if (mode == C3_PLAIN) BRP_LAUNCH((pass3_cplx_kernel<n, kRows3, C3_PLAIN>), grid, block, 0, s, a);     \
    else if (mode == C3_MULCONJ) BRP_LAUNCH((pass3_cplx_kernel<n, kRows3, C3_MULCONJ>), grid, block, 0, s, a); \
    else BRP_LAUNCH((pass3_cplx_kernel<n, kRows3, C3_CHIRP>), grid, block, 0, s, a);                     \
    break;                                                                                                         \
  }
    BRP_P3_LENGTHS(X)
#undef X
    default: return hipErrorInvalidValue;
  }
  return launch_status();
}

bool chirp_rev_supported(const FFTPlan3& plan) {
  bool l1 = false, l2 = false, l3 = false;
  switch (plan.L1) {
#define X(n) case n:
    BRP_P1G_LENGTHS(X)
#undef X
    l1 = true;
    default: break;
  }
  switch (plan.L2) {
#define X(n) case n:
    BRP_P2R_LENGTHS(X) BRP_P2G_LENGTHS(X)
#undef X
    l2 = true;
    default: break;
  }
  switch (plan.L3) {
#define X(n) case n:
    BRP_P3_LENGTHS(X)
#undef X
    l3 = true;
    default: break;
  }
  return l1 && l2 && l3 && BRP_P1G;
}

// rows per pass3_mid workgroup: 8 (measured best: -P 2.7 3 151 vs 2 683
// templates/s with whole-wave workgroups of 16 rows for L3 = 320, and 2 901
// for a register-staged row FFT, round 5); a.whole_waves: 16 or 32 rows where
// 8 rows of L / 16 threads are not whole waves (A/B switch)
template <int L>
constexpr int mid_rows() {
  return (8 * tpc_for<L>()) % kWave == 0 ? 8 : (16 * tpc_for<L>()) % kWave == 0 ? 16 : 32;
}

hipError_t launch_pass3_mid(const FFTPlan3& plan, const Pass3MidArgs& a, int batch, hipStream_t s) {
  const uint32_t rows = plan.L1 * plan.L2;
  switch (plan.L3) {
#define X(n)                                                                                              \
  case n: {                                                                                               \
    constexpr int R = mid_rows<n>();                                                                      \
    if (!a.whole_waves || R == 8) {                                                                       \
      if (rows % 8 != 0) return hipErrorInvalidValue;                                                     \
      BRP_LAUNCH((pass3_mid_kernel<n, 8>), dim3(rows / 8, batch), dim3(8 * tpc_for<n>()), 0, s, a); \
    } else {                                                                                              \
      if (rows % R != 0) return hipErrorInvalidValue;                                                     \
      BRP_LAUNCH((pass3_mid_kernel<n, R>), dim3(rows / R, batch), dim3(R * tpc_for<n>()), 0, s, a); \
    }                                                                                                     \
    break;                                                                                                \
  }
    BRP_P3_LENGTHS(X)
#undef X
    default: return hipErrorInvalidValue;
  }
  return launch_status();
}

// the module's code object onto the current device (loaded lazily at the
// first launch otherwise: ~14 ms inside the first template batch, round 6)
hipError_t preload_fft_passes() {
  hipFuncAttributes at;
  return hipFuncGetAttributes(&at, reinterpret_cast<const void*>(&pass3_kernel<256, kRowsP, P3_POWER>));
}

hipError_t launch_pass3_plain(const FFTPlan3& plan, const Pass3PlainArgs& a, hipStream_t s) {
  const dim3 grid(plan.wg3_plain());
  switch (plan.L3) {
#define X(n)                                                                                       \
  case n:                                                                                          \
    BRP_LAUNCH((pass3_plain_kernel<n, kRows3>), grid, dim3(kRows3 * tpc_for<n>()), 0, s, a); \
    break;
    BRP_P3_LENGTHS(X)
#undef X
    default: return hipErrorInvalidValue;
  }
  return launch_status();
}

}  // namespace hipk
}  // namespace brp
