// Chirp-z (Bluestein) kernels for FFT lengths outside the smooth set (see
// bluestein_kernels.hpp). The convolution itself runs on the three-pass FFT
// (fft_passes.hip); these kernels produce its chirp-multiplied input and
// consume its output.
#include "bluestein_kernels.hpp"
#include "fft_block.hpp"

namespace brp {
namespace hipk {

namespace {

constexpr int kThreads = 256;
constexpr int kPerThread = 4;  // outputs per thread of the chirp-in kernel

__device__ __forceinline__ float2 chirp_w(const TwiddleTable& t, uint32_t n) {
  return tw_lookup(t, static_cast<uint64_t>(n) * n);  // W_{2Mb}^{n^2 mod 2Mb}
}

template <int MODE>
__global__ void __launch_bounds__(kThreads) bs_chirp_in_kernel(BsInArgs a) {
  const int b = blockIdx.y;
  float2* y = a.y + static_cast<size_t>(b) * a.L;
  const uint32_t n0 = (blockIdx.x * kPerThread) * kThreads + threadIdx.x;
#pragma unroll
  for (int u = 0; u < kPerThread; ++u) {
    const uint32_t n = n0 + u * kThreads;
    if (n >= a.L) break;
    float2 v = make_float2(0.0f, 0.0f);
    if (MODE == BS_IN_HCHIRP) {
      // h_n = conj(w_n) for n < Mb, h_{L-n} = conj(w_n) for 0 < n < Mb
      if (n < a.Mb) v = conjf2(chirp_w(a.chirp, n));
      else if (a.L - n < a.Mb) v = conjf2(chirp_w(a.chirp, a.L - n));
    } else if (n < a.Mb) {
      float2 x;
      if (MODE == BS_IN_REAL2) {
        x = make_float2(2 * n < a.n_real ? BRP_LD(&a.real_in[2 * n]) : 0.0f,
                       2 * n + 1 < a.n_real ? BRP_LD(&a.real_in[2 * n + 1]) : 0.0f);
      } else if (MODE == BS_IN_REAL1) {
        x = make_float2(n < a.n_real ? BRP_LD(&a.real_in[n]) : 0.0f, 0.0f);
      } else if (MODE == BS_IN_CONJ) {
        x = conjf2(BRP_LD(&a.cplx_in[n]));
      } else {  // BS_IN_HERM_CONJ: F_n = X_n (n <= (N-1)/2), conj(X_{N-n}) above; input conj(F_n)
        // with the whitening's zeroed edges and Im X_0 = 0 (c2r semantics, as tangle_kernel)
        auto bin = [&](uint32_t q) -> float2 {
          if (q < a.w2 || q >= a.fft_size - a.w2) return make_float2(0.0f, 0.0f);
          float2 v = BRP_LD(&a.cplx_in[q]);
          if (q == 0) v.y = 0.0f;
          return v;
        };
        const uint32_t half = (a.nsamples - 1) / 2;
        x = n <= half ? conjf2(bin(n)) : bin(a.nsamples - n);
      }
      v = cmul(x, chirp_w(a.chirp, n));
    }
    BRP_ST(&y[n], v);
  }
}

// X_k of the real transform from the length-Mb DFT A: even N (A = DFT of the
// packed pairs, Mb = N/2): untangle A_k, A_{Mb-k}; odd N (A = DFT of the real
// series, Mb = N): X_k = A_k for k <= (N-1)/2 and the DFT's own symmetric value
// conj(A_{N-k}) at k = (N+1)/2 (the one bin fft_size reaches beyond it)
__device__ __forceinline__ float2 bs_bin(const float2* A, uint32_t Mb, uint32_t N, const TwiddleTable& tw, uint32_t k) {
  if (N & 1u) {
    const uint32_t half = (N - 1) / 2;
    return k <= half ? BRP_LD(&A[k]) : conjf2(BRP_LD(&A[N - k]));
  }
  if (k == Mb) {  // Nyquist
    const float2 a0 = BRP_LD(&A[0]);
    return make_float2(a0.x - a0.y, 0.0f);
  }
  const float2 zk = BRP_LD(&A[k]), zm = BRP_LD(&A[(Mb - k) % Mb]);
  return untangle_w(zk, zm, tw_lookup(tw, 2ull * k));  // W_N^k = W_2N^{2k}
}

// Each thread handles kPowBins bins k (kThreads apart): W_2N^k and W_2N^{n_s k}
// (the padding correction) are looked up exactly for the first and stepped by
// one complex product per bin after it (one 64-bit reduction and table pair
// per kPowBins bins instead of two per bin: n_s k mod 2N lands anywhere in the
// table). A wave's loads and stores cover 64 consecutive bins.
// Measured (one call, templates/s at -P 2.7 / 2.9 / 1.1): 4 contiguous bins
// 3 719 / 3 756 / 9 804, 8 contiguous 3 518 / 3 164 / 9 212, 4 strided
// 3 810 / 3 956 / 10 149, 8 strided 3 865 / 3 980 / 10 171 (default)
#ifndef BRP_POW_BINS
#define BRP_POW_BINS 8
#endif
#ifndef BRP_POW_STRIDED
#define BRP_POW_STRIDED 1
#endif
constexpr int kPowBins = BRP_POW_BINS;
// strided form: the thread's bins are kThreads apart (every load and store
// instruction of a wave covers 64 consecutive bins)
constexpr bool kPowStrided = BRP_POW_STRIDED != 0;
constexpr uint32_t kPowStep = kPowStrided ? kThreads : 1;

template <bool HALF>
__global__ void __launch_bounds__(kThreads) bs_power_kernel(BsPowerArgs a) {
  const int b = blockIdx.y;  // transform
  const uint32_t k0 = kPowStrided ? blockIdx.x * kThreads * kPowBins + threadIdx.x
                                  : (blockIdx.x * kThreads + threadIdx.x) * kPowBins;
  if (k0 >= a.limit) return;
  const uint32_t real_bins = a.nsamples / 2 + 1;  // bins the real DFT defines
  const float2* A = a.A + static_cast<size_t>(b) * a.L;
  // per template: W_2N^{k0}, W_2N^{n_s k0} and their per-bin steps
  struct Walk {
    float2 tk, ta, sk, sa;
    float dS;
    uint32_t n_s;
  };
  auto walk = [&](uint32_t t) {
    Walk w{};
    w.n_s = BRP_LD(&a.tmpl[t]).n_steps;
    if (w.n_s > 0) {
      w.dS = static_cast<float>(BRP_LD(&a.delta[t]));
      w.tk = tw_lookup(a.tw, k0);
      w.sk = tw_lookup(a.tw, kPowStep);
      w.ta = tw_lookup(a.tw, static_cast<uint64_t>(w.n_s) * k0);
      w.sa = tw_lookup(a.tw, static_cast<uint64_t>(w.n_s) * kPowStep);
    }
    return w;
  };
  // X_k (+ delta * S_k, S_k the transform of the padding indicator) -> |.|^2 / N
  auto power = [&](float2 x, const Walk& w) {
    if (w.n_s > 0) {
      const float2 sp = padding_spectrum_t(w.ta, w.tk, cmul(w.ta, conjf2(w.tk)));  // tc = W_2N^{(n_s - 1) k}
      x = make_float2(x.x + w.dS * sp.x, x.y + w.dS * sp.y);
    }
    return (x.x * x.x + x.y * x.y) * a.norm;
  };
  auto advance = [](Walk& w) {
    if (w.n_s > 0) {
      w.tk = cmul(w.tk, w.sk);
      w.ta = cmul(w.ta, w.sa);
    }
  };
  auto store = [&](uint32_t t, uint32_t k, float p) {
    const size_t o = static_cast<size_t>(t) * a.ps_stride + k;
    if (HALF) BRP_ST(&a.ps16[o], static_cast<_Float16>(fminf(p, 65504.0f)));  // saturate: no inf in the fp16 spectrum
    else BRP_ST(&a.ps[o], p);
  };
  if (!a.pair) {
    Walk w = walk(b);
#pragma unroll
    for (int i = 0; i < kPowBins; ++i) {
      const uint32_t k = k0 + i * kPowStep;
      if (k >= a.limit) break;
      const bool live = k > 0 && k < real_bins;
      store(b, k, live ? power(bs_bin(A, a.Mb, a.nsamples, a.tw, k), w) : 0.0f);
      advance(w);
    }
    return;
  }
  // odd N, A = DFT of x_a + i x_b: X_a = (A_k + conj A_{N-k}) / 2, X_b = -i (A_k - conj A_{N-k}) / 2
  const uint32_t ta = 2 * b, tb = 2 * b + 1;
  const bool has_b = tb < a.n_tmpl;
  Walk wa = walk(ta), wb = has_b ? walk(tb) : Walk{};
#pragma unroll
  for (int i = 0; i < kPowBins; ++i) {
    const uint32_t k = k0 + i * kPowStep;
    if (k >= a.limit) break;
    const bool live = k > 0 && k < real_bins;
    float pa = 0.0f, pb = 0.0f;
    if (live) {
      const float2 ak = BRP_LD(&A[k]), am = conjf2(BRP_LD(&A[a.nsamples - k]));
      pa = power(make_float2(0.5f * (ak.x + am.x), 0.5f * (ak.y + am.y)), wa);
      if (has_b) pb = power(make_float2(0.5f * (ak.y - am.y), -0.5f * (ak.x - am.x)), wb);
    }
    store(ta, k, pa);
    if (has_b) store(tb, k, pb);
    advance(wa);
    advance(wb);
  }
}

__global__ void __launch_bounds__(kThreads) bs_spec_kernel(const float2* A, uint32_t Mb, uint32_t N, TwiddleTable tw,
                                                           uint32_t fft_size, float2* spec) {
  const uint32_t k = blockIdx.x * kThreads + threadIdx.x;
  if (k < fft_size) BRP_ST(&spec[k], bs_bin(A, Mb, N, tw, k));
}

// inverse transforms: A = DFT(conj(input)); even N: the packed pairs
// conj(A_n) -> (x[2n], x[2n+1]); odd N: x[n] = Re A_n
__global__ void __launch_bounds__(kThreads) bs_real_out_kernel(const float2* A, uint32_t Mb, uint32_t N, float scale,
                                                               float* out, uint32_t n_out) {
  const uint32_t n = blockIdx.x * kThreads + threadIdx.x;
  if (n >= Mb) return;
  const float2 v = BRP_LD(&A[n]);
  if (N & 1u) {
    if (n < n_out) BRP_ST(&out[n], v.x * scale);
  } else {
    if (2 * n < n_out) BRP_ST(&out[2 * n], v.x * scale);
    if (2 * n + 1 < n_out) BRP_ST(&out[2 * n + 1], -v.y * scale);
  }
}

// H in the row layout of the transposed convolution (Pass3MidArgs):
// hp[(k1 L2 + k2) L3 + k3] = H[k1 + L1 k2 + L1 L2 k3] (once per plan)
__global__ void __launch_bounds__(kThreads) bs_rows_kernel(const float2* H, float2* hp, uint32_t L1, uint32_t L2,
                                                           uint32_t L3) {
  const uint32_t i = blockIdx.x * kThreads + threadIdx.x;
  if (i >= L1 * L2 * L3) return;
  const uint32_t row = i / L3, k3 = i % L3;
  const uint32_t k1 = row / L2, k2 = row % L2;
  BRP_ST(&hp[i], BRP_LD(&H[k1 + L1 * k2 + L1 * L2 * k3]));
}

}  // namespace

hipError_t preload_bluestein() {
  hipFuncAttributes at;
  return hipFuncGetAttributes(&at, reinterpret_cast<const void*>(&bs_rows_kernel));
}

hipError_t launch_bs_rows(const float2* H, float2* hp, uint32_t L1, uint32_t L2, uint32_t L3, hipStream_t s) {
  const uint32_t n = L1 * L2 * L3;
  BRP_LAUNCH(bs_rows_kernel, dim3((n + kThreads - 1) / kThreads), dim3(kThreads), 0, s, H, hp, L1, L2, L3);
  return launch_status();
}

uint32_t bs_chirp_in_blocks(uint32_t L) { return (L + kThreads * kPerThread - 1) / (kThreads * kPerThread); }

hipError_t launch_bs_chirp_in(BsInMode mode, const BsInArgs& a, int batch, uint32_t* n_partials, hipStream_t s) {
  const dim3 grid(bs_chirp_in_blocks(a.L), batch);
  if (n_partials) *n_partials = grid.x;
  switch (mode) {
#define BRP_BS_CASE(M) \
  case M: BRP_LAUNCH((bs_chirp_in_kernel<M>), grid, dim3(kThreads), 0, s, a); break;
    BRP_BS_CASE(BS_IN_REAL2)
    BRP_BS_CASE(BS_IN_REAL1)
    BRP_BS_CASE(BS_IN_CONJ)
    BRP_BS_CASE(BS_IN_HERM_CONJ)
    BRP_BS_CASE(BS_IN_HCHIRP)
#undef BRP_BS_CASE
    default: return hipErrorInvalidValue;
  }
  return launch_status();
}

hipError_t launch_bs_power(const BsPowerArgs& a, int batch, hipStream_t s) {
  const dim3 grid((a.limit + kThreads * kPowBins - 1) / (kThreads * kPowBins), batch);
  if (a.ps16) BRP_LAUNCH((bs_power_kernel<true>), grid, dim3(kThreads), 0, s, a);
  else BRP_LAUNCH((bs_power_kernel<false>), grid, dim3(kThreads), 0, s, a);
  return launch_status();
}

hipError_t launch_bs_spec(const float2* A, uint32_t Mb, uint32_t nsamples, const TwiddleTable& tw, uint32_t fft_size,
                          float2* spec, hipStream_t s) {
  BRP_LAUNCH(bs_spec_kernel, dim3((fft_size + kThreads - 1) / kThreads), dim3(kThreads), 0, s, A, Mb,
                     nsamples, tw, fft_size, spec);
  return launch_status();
}

hipError_t launch_bs_real_out(const float2* A, uint32_t Mb, uint32_t nsamples, float scale, float* out,
                              uint32_t n_out, hipStream_t s) {
  BRP_LAUNCH(bs_real_out_kernel, dim3((Mb + kThreads - 1) / kThreads), dim3(kThreads), 0, s, A, Mb, nsamples,
                     scale, out, n_out);
  return launch_status();
}

}  // namespace hipk
}  // namespace brp
