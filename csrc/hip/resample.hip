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
  if (reset != nullptr && blockIdx.x == 0 && threadIdx.x == 0) BRP_ST(reset, 0u);
  TemplateDev& td = tmpl[blockIdx.x];
  const ResampParams p = BRP_LD(&td).p;
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
  if (threadIdx.x == 0) BRP_ST(&td.n_steps, best);
}

__global__ void resample_kernel(const float* series, uint32_t n_unpadded, const TemplateDev* tmpl, float* out,
                                uint32_t nsamples) {
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= nsamples) return;
  const TemplateDev td = BRP_LD(tmpl);
  float v = 0.0f;
  if (m < td.n_steps) {
    const float d = resamp_del_t(m, td.p, kSinLut, kCosLut);
    int idx = resamp_nearest(m, d);
    idx = idx < 0 ? 0 : (idx >= static_cast<int>(n_unpadded) ? static_cast<int>(n_unpadded) - 1 : idx);
    v = BRP_LD(&series[idx]);
  }
  BRP_ST(&out[m], v);
}

}  // namespace

hipError_t preload_resample() {
  hipFuncAttributes at;
  return hipFuncGetAttributes(&at, reinterpret_cast<const void*>(&nsteps_kernel));
}

hipError_t launch_nsteps(TemplateDev* tmpl, int batch, hipStream_t s, uint32_t* reset) {
  BRP_LAUNCH(nsteps_kernel, dim3(batch), dim3(kThreads), 0, s, tmpl, reset);
  return launch_status();
}

hipError_t launch_resample(const float* series, uint32_t n_unpadded, const TemplateDev* tmpl, float* out,
                           uint32_t nsamples, hipStream_t s) {
  BRP_LAUNCH(resample_kernel, dim3((nsamples + 255) / 256), dim3(256), 0, s, series, n_unpadded, tmpl, out,
                     nsamples);
  return launch_status();
}

}  // namespace hipk
}  // namespace brp
