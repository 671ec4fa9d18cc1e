// Device kernels of the whitening / RFI-zapping step (implementation: whiten.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "hip_common.hpp"

namespace brp {
namespace hipk {

hipError_t launch_whiten_power(const float2* spec, uint32_t n, float* ps, hipStream_t s);
// WU payload -> floats exactly as the host reader (demod_binary.c:830-842,
// io.cpp): 4-bit high nibble first, (float)((double)v / scale); 8-bit signed
hipError_t launch_unpack(const uint8_t* packed, uint32_t n_packed, bool four_bit, double scale, float* out,
                         uint32_t n_out, hipStream_t s);
bool running_median_supported(uint32_t W);
hipError_t launch_running_median(const float* in, uint32_t n_in, uint32_t W, float* med, hipStream_t s);
// any window (used above running_median_supported's limit): global radix sort
// + per-run median pointer walk (rmed_wide.hip); scratch of
// running_median_wide_scratch_bytes(n_in) bytes
size_t running_median_wide_scratch_bytes(uint32_t n_in);
hipError_t launch_running_median_wide(const float* in, uint32_t n_in, uint32_t W, float* med, void* scratch,
                                      hipStream_t s);
hipError_t launch_whiten_scale(float2* spec, const float* med, uint32_t white_size, uint32_t w2, hipStream_t s);
hipError_t launch_zap(float2* spec, uint32_t fft_size, const uint32_t* bins, const float2* noise, uint32_t n,
                      hipStream_t s);
hipError_t launch_tangle(const float2* spec, uint32_t M, uint32_t fft_size, uint32_t w2, const TwiddleTable& tw,
                         float2* z, hipStream_t s);

}  // namespace hipk
}  // namespace brp
