// Resampling helpers that are not fused into the FFT: the per-template series
// length and a stand-alone resampler used by tests / debugging.
//
// n_steps replaces the reference's single-thread backwards scan
// (cuda/app/demod_binary_cuda.cuh:83-96, launched 1x1 followed by a blocking
// device->host copy, demod_binary_cuda.cu:516-560): one workgroup per template
// evaluates the end condition over the whole tail window that |del_t| can reach
// and takes the largest index that is kept. The result stays on the device.
#include "fft_kernels.hpp"
#include "resample_kernels.hpp"

namespace brp {
namespace hipk {

namespace {

constexpr int kThreads = 256;

__global__ void __launch_bounds__(kThreads) nsteps_kernel(TemplateDev* tmpl, uint32_t* reset) {
  __shared__ uint32_t best;
  if (reset != nullptr && blockIdx.x == 0 && threadIdx.x == 0) *reset = 0;
  TemplateDev& td = tmpl[blockIdx.x];
  const ResampParams p = td.p;
  const uint32_t nu = p.nsamples_unpadded;
  // |del_t| <= |tau*step_inv| + |S0| (+ LUT error); scan that tail plus margin
  const float reach = fabsf(p.tau * p.step_inv) + fabsf(p.S0) + 4.0f;
  uint32_t span = static_cast<uint32_t>(fminf(reach, static_cast<float>(nu - 1))) + 2;
  if (span > nu) span = nu;
  if (threadIdx.x == 0) best = 0;
  __syncthreads();
  uint32_t local = 0;
  bool found = false;
  for (uint32_t t = threadIdx.x; t < span; t += kThreads) {
    const uint32_t m = nu - 1 - t;
    const float dt = resamp_del_t(m, p, kSinLut, kCosLut);
    if (!resamp_beyond_end(m, dt, nu)) {
      if (!found || m > local) local = m;
      found = true;
    }
  }
  if (found) atomicMax(&best, local);
  __syncthreads();
  if (threadIdx.x == 0) td.n_steps = best;
}

__global__ void resample_kernel(const float* series, uint32_t n_unpadded, const TemplateDev* tmpl, float* out,
                                uint32_t nsamples) {
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= nsamples) return;
  const TemplateDev td = *tmpl;
  float v = 0.0f;
  if (m < td.n_steps) {
    const float d = resamp_del_t(m, td.p, kSinLut, kCosLut);
    int idx = resamp_nearest(m, d);
    idx = idx < 0 ? 0 : (idx >= static_cast<int>(n_unpadded) ? static_cast<int>(n_unpadded) - 1 : idx);
    v = series[idx];
  }
  out[m] = v;
}

// 4 consecutive samples per thread and step (one float4 store), the
// workgroup's chunk a multiple of 1024 samples; all 4 gathers in flight together
__global__ void __launch_bounds__(kThreads) resample_centred_kernel(ResampCentredArgs a) {
  __shared__ float lut_s[kLutSize], lut_c[kLutSize];
  __shared__ double red[kThreads / kWave + 1];
  for (int i = threadIdx.x; i < kLutSize; i += kThreads) {
    lut_s[i] = kSinLut[i];
    lut_c[i] = kCosLut[i];
  }
  __syncthreads();
  const uint32_t t = blockIdx.y;
  const TemplateDev td = a.tmpl[t];
  const float* series = a.series + static_cast<size_t>(td.wu) * a.n_unpadded;
  float* y = a.y + static_cast<size_t>(t) * a.ystride;
  const bool fast = a.n_unpadded <= (1u << 23);
  const int last = static_cast<int>(a.n_unpadded) - 1;
  const uint32_t chunk = ((a.n_out + gridDim.x - 1) / gridDim.x + 1023) / 1024 * 1024;
  const uint32_t lo = blockIdx.x * chunk, hi = min(lo + chunk, a.n_out);
  float fsum = 0.0f;
  for (uint32_t m0 = lo + 4 * threadIdx.x; m0 < hi; m0 += 4 * kThreads) {
    int idx[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const uint32_t m = m0 + e;
      int i = -1;
      if (m < td.n_steps && m < hi) {
        const float dt = resamp_del_t(m, td.p, lut_s, lut_c);
        i = min(max(fast ? resamp_nearest_f(m, dt) : resamp_nearest(m, dt), 0), last);
      }
      idx[e] = i;
    }
    float raw[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) raw[e] = series[idx[e] < 0 ? 0 : idx[e]];
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[e] = idx[e] < 0 ? 0.0f : raw[e] - td.mu0;
      fsum += v[e];
    }
    if (m0 + 4 <= a.ystride) *reinterpret_cast<float4*>(y + m0) = make_float4(v[0], v[1], v[2], v[3]);
  }
  double sum = wave_sum(static_cast<double>(fsum));
  if (threadIdx.x % kWave == 0) red[threadIdx.x / kWave] = sum;
  __syncthreads();
  if (threadIdx.x == 0) {
    double tot = 0.0;
    for (int w = 0; w < kThreads / kWave; ++w) tot += red[w];
    a.partials[static_cast<size_t>(t) * a.n_partials + blockIdx.x] = tot;
  }
}

}  // namespace

hipError_t launch_resample_centred(const ResampCentredArgs& a, int templates, hipStream_t s) {
  if (a.ystride % 4 != 0 || a.ystride < a.n_out) return hipErrorInvalidValue;
  hipLaunchKernelGGL(resample_centred_kernel, dim3(a.n_partials, templates), dim3(kThreads), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_nsteps(TemplateDev* tmpl, int batch, hipStream_t s, uint32_t* reset) {
  hipLaunchKernelGGL(nsteps_kernel, dim3(batch), dim3(kThreads), 0, s, tmpl, reset);
  return hipGetLastError();
}

hipError_t launch_resample(const float* series, uint32_t n_unpadded, const TemplateDev* tmpl, float* out,
                           uint32_t nsamples, hipStream_t s) {
  hipLaunchKernelGGL(resample_kernel, dim3((nsamples + 255) / 256), dim3(256), 0, s, series, n_unpadded, tmpl, out,
                     nsamples);
  return hipGetLastError();
}

}  // namespace hipk
}  // namespace brp
