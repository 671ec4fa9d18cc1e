#pragma once

#include <hip/hip_runtime.h>

#include "fft_kernels.hpp"

namespace brp {
namespace hipk {

// n_steps of every template of a batch (written into tmpl[b].n_steps); also
// zeroes *reset (the batch's candidate counter) when given
hipError_t launch_nsteps(TemplateDev* tmpl, int batch, hipStream_t s, uint32_t* reset = nullptr);
// stand-alone resampling (zero beyond n_steps) for tests / debugging
hipError_t launch_resample(const float* series, uint32_t n_unpadded, const TemplateDev* tmpl, float* out,
                           uint32_t nsamples, hipStream_t s);

}  // namespace hipk
}  // namespace brp
