// Whitening + RFI zapping kernels (reference demod_binary.c:857-1079, done on the
// host with FFTW/rngmed/GSL there; on MI355X it runs on the device between a
// forward and an inverse pass of the same hand-written FFT).
#include "hip_common.hpp"
#include "whiten_kernels.hpp"

namespace brp {
namespace hipk {

namespace {

__global__ void whiten_power_kernel(const float2* spec, uint32_t n, float* ps) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  float p = 0.0f;
  if (k != 0) {
    const double re = spec[k].x, im = spec[k].y;
    p = static_cast<float>(re * re + im * im);
  }
  ps[k] = p;
}

// Exact running median: each workgroup sorts (value, position) of its span in
// LDS (bitonic) and every thread walks the sorted span counting the entries of
// its own window up to the middle order statistics.
template <int SPAN>
__global__ void __launch_bounds__(1024) running_median_kernel(const float* in, uint32_t n_in, uint32_t W,
                                                              float* med, uint32_t n_out, uint32_t per_block) {
  __shared__ float key[SPAN];
  __shared__ uint32_t pos[SPAN];
  const uint32_t o0 = blockIdx.x * per_block;
  for (int t = threadIdx.x; t < SPAN; t += blockDim.x) {
    const uint32_t g = o0 + t;
    key[t] = (t < static_cast<int>(per_block + W - 1) && g < n_in) ? in[g] : __builtin_inff();
    pos[t] = t;
  }
  __syncthreads();
  // bitonic sort ascending by (key, pos)
  for (int size = 2; size <= SPAN; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = threadIdx.x; t < SPAN / 2; t += blockDim.x) {
        const int lo = 2 * t - (t & (stride - 1));
        const int hi = lo + stride;
        const bool asc = ((lo & size) == 0);
        const float ka = key[lo], kb = key[hi];
        const uint32_t pa = pos[lo], pb = pos[hi];
        const bool gt = (ka > kb) || (ka == kb && pa > pb);
        if (gt == asc) {
          key[lo] = kb;
          key[hi] = ka;
          pos[lo] = pb;
          pos[hi] = pa;
        }
      }
      __syncthreads();
    }
  }
  const uint32_t mid = (W + (W & 1)) / 2 - 1;
  const bool odd = (W & 1) != 0;
  for (uint32_t t = threadIdx.x; t < per_block; t += blockDim.x) {
    const uint32_t o = o0 + t;
    if (o >= n_out) break;
    uint32_t cnt = 0;
    float a = 0.0f, bval = 0.0f;
    bool have_a = false;
    for (int e = 0; e < SPAN; ++e) {
      const uint32_t p = pos[e];
      if (p >= t && p < t + W) {
        if (cnt == mid) {
          a = key[e];
          have_a = true;
          if (odd) break;
        } else if (cnt == mid + 1) {
          bval = key[e];
          break;
        }
        ++cnt;
      }
    }
    (void)have_a;
    med[o] = odd ? a : static_cast<float>(static_cast<double>(a + bval) / 2.0);
  }
}

// spec[w2 + i] *= sqrt(ln2 / med[i]) for i < white_size
__global__ void whiten_scale_kernel(float2* spec, const float* med, uint32_t white_size, uint32_t w2) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= white_size) return;
  const float f = static_cast<float>(sqrt(M_LN2 / static_cast<double>(med[i])));
  float2 v = spec[i + w2];
  v.x *= f;
  v.y *= f;
  spec[i + w2] = v;
}

__global__ void zap_kernel(float2* spec, uint32_t fft_size, const uint32_t* bins, const float2* noise, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t k = bins[i];
  if (k < fft_size) spec[k] = noise[i];
}

// Inverse real-FFT packing: Z_k = (X_k + conj X_{M-k}) + i W_N^{-k} (X_k - conj X_{M-k}),
// with the first/last w2 bins zeroed and Im X_0 = Im X_M = 0 (FFTW c2r semantics).
__global__ void tangle_kernel(const float2* spec, uint32_t M, uint32_t fft_size, uint32_t w2, TwiddleTable tw,
                              float2* z) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= M) return;
  auto bin = [&](uint32_t q) -> float2 {
    if (q < w2 || q >= fft_size - w2) return make_float2(0.0f, 0.0f);
    float2 v = spec[q];
    if (q == 0 || q == M) v.y = 0.0f;
    return v;
  };
  const float2 a = bin(k);
  const float2 bc = conjf2(bin(M - k));
  const float2 w = conjf2(tw_lookup32(tw, 2u * k));  // W_N^{-k}
  const float2 d = csub(a, bc);
  const float2 iwd = cmul(make_float2(0.0f, 1.0f), cmul(w, d));
  z[k] = cadd(cadd(a, bc), iwd);
}

}  // namespace

hipError_t launch_whiten_power(const float2* spec, uint32_t n, float* ps, hipStream_t s) {
  hipLaunchKernelGGL(whiten_power_kernel, dim3((n + 255) / 256), dim3(256), 0, s, spec, n, ps);
  return hipGetLastError();
}

bool running_median_supported(uint32_t W) { return W >= 1 && W <= 3072; }

hipError_t launch_running_median(const float* in, uint32_t n_in, uint32_t W, float* med, hipStream_t s) {
  if (!running_median_supported(W) || n_in < W) return hipErrorInvalidValue;
  const uint32_t n_out = n_in - W + 1;
  if (W <= 1024) {
    constexpr int kSpan = 2048;
    const uint32_t per = kSpan - W + 1;
    hipLaunchKernelGGL((running_median_kernel<kSpan>), dim3((n_out + per - 1) / per), dim3(1024), 0, s, in, n_in, W,
                       med, n_out, per);
  } else {
    constexpr int kSpan = 4096;
    const uint32_t per = kSpan - W + 1;
    hipLaunchKernelGGL((running_median_kernel<kSpan>), dim3((n_out + per - 1) / per), dim3(1024), 0, s, in, n_in, W,
                       med, n_out, per);
  }
  return hipGetLastError();
}

hipError_t launch_whiten_scale(float2* spec, const float* med, uint32_t white_size, uint32_t w2, hipStream_t s) {
  hipLaunchKernelGGL(whiten_scale_kernel, dim3((white_size + 255) / 256), dim3(256), 0, s, spec, med, white_size, w2);
  return hipGetLastError();
}

hipError_t launch_zap(float2* spec, uint32_t fft_size, const uint32_t* bins, const float2* noise, uint32_t n,
                      hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(zap_kernel, dim3((n + 255) / 256), dim3(256), 0, s, spec, fft_size, bins, noise, n);
  return hipGetLastError();
}

hipError_t launch_tangle(const float2* spec, uint32_t M, uint32_t fft_size, uint32_t w2, const TwiddleTable& tw,
                         float2* z, hipStream_t s) {
  hipLaunchKernelGGL(tangle_kernel, dim3((M + 255) / 256), dim3(256), 0, s, spec, M, fft_size, w2, tw, z);
  return hipGetLastError();
}

}  // namespace hipk
}  // namespace brp
