#pragma once

#include <hip/hip_runtime.h>

#include "fft_kernels.hpp"

namespace brp {
namespace hipk {

// n_steps of every template of a batch (written into tmpl[b].n_steps); also
// zeroes *reset (the batch's candidate counter) when given
hipError_t launch_nsteps(TemplateDev* tmpl, int batch, hipStream_t s, uint32_t* reset = nullptr);
// Centred resampled series of a launch group's templates for the chirp-z
// pass 1 (Pass1Args::y): y[t][m] = series[nearest(m)] - mu0 for m < n_steps,
// 0 for n_steps <= m < n_out; one double partial sum of the centred samples
// per workgroup into partials[t][blockIdx.x] (grid.x = n_partials, what pass
// 2 reduces into the mean-padding delta)
struct ResampCentredArgs {
  const float* series;         // [slots][n_unpadded]
  uint32_t n_unpadded;
  const TemplateDev* tmpl;     // [templates]
  float* y;                    // [templates][ystride]
  uint32_t ystride, n_out;
  double* partials;            // [templates][n_partials]
  uint32_t n_partials;
};
hipError_t launch_resample_centred(const ResampCentredArgs& a, int templates, hipStream_t s);
// stand-alone resampling (zero beyond n_steps) for tests / debugging
hipError_t launch_resample(const float* series, uint32_t n_unpadded, const TemplateDev* tmpl, float* out,
                           uint32_t nsamples, hipStream_t s);

}  // namespace hipk
}  // namespace brp
