// Two-pass template FFT of the production shape (implementation: fft2.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "fft_kernels.hpp"

namespace brp {
namespace hipk {

constexpr uint32_t kFft2L1 = 768;   // column-pass length (3 * 16 * 16)
constexpr uint32_t kFft2R = 8192;   // row length (16 * 16 * 16 * 2)
constexpr uint32_t kFft2M = kFft2L1 * kFft2R;  // 6 291 456 = N/2 for N = 3 * 2^22

// pass A: resampling gather + 768-point column FFTs
struct ColAArgs {
  float2* out;                 // [batch][M]: row k1 (R complex) contiguous
  uint32_t M;
  const float* series;         // [slots][n_unpadded]
  uint32_t n_unpadded;
  const TemplateDev* tmpl;     // [batch]
  double* partials;            // [batch][R / 16] sums of (sample - mu0)
  TwiddleTable tw;             // W_4M^e
  const float2* w768;          // W_768^e, e < 768
  uint32_t* reset;             // zeroed by workgroup (0, 0) when non-null (the batch's candidate counter)
};

// pass B: 8192-point row FFTs of row pairs + untangle + power spectrum (slab-major)
struct RowBArgs {
  const float2* buf;           // [batch][M] from pass A
  uint32_t M;
  TwiddleTable tw;
  const float2* t256;          // W_256^e
  const float2* t4096;         // W_4096: lo[64] | hi[64]
  const float2* t8192;         // W_8192: lo[64] | hi[64]
  uint32_t limit;              // bins k < limit only
  float* pss;                  // [batch][pss_stride], PSs[k1 * R + m] = PS[k1 + 768 m]
  uint32_t pss_stride;
  float norm;                  // 1/N
  const TemplateDev* tmpl;     // n_steps
  const double* partials;      // pass A sums, reduced in a fixed order by every workgroup
  uint32_t n_partials;         // per template
  // Nyquist bin M (natural order, when M < limit)
  float* ps;
  _Float16* ps16;
  uint32_t ps_stride;
};

// slab-major -> natural-order power spectrum
struct PsTArgs {
  const float* pss;
  uint32_t pss_stride;
  float* ps;                   // natural order [batch][ps_stride] (or ps16)
  _Float16* ps16;
  uint32_t ps_stride;
  uint32_t limit, M;
};

hipError_t launch_colA(const ColAArgs& a, int batch, hipStream_t s);
hipError_t launch_rowB(const RowBArgs& a, int batch, hipStream_t s);
hipError_t launch_psT(const PsTArgs& a, int batch, hipStream_t s);

}  // namespace hipk
}  // namespace brp
