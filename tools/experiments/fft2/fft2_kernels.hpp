// Two-pass template FFT of the production shape (implementation: fft2.hip).
//
// N = 3 * 2^22 real samples (the 2^22-sample work unit, padding 3), packed as
// M = N/2 = 768 * 8192 complex points, n = n1 * R + n' (n1 < 768, n' < R = 8192),
// k = k1 + 768 m:
//   X[k1 + 768 m] = sum_n' W_R^{n' m} W_M^{n' k1} sum_n1 z[n1 R + n'] W_768^{n1 k1}
// pass A: resampling gather + 768-point column DFTs over n1 (+ W_M^{n' k1}),
//         row k1 (R points) written contiguously;
// pass B: 8192-point FFTs of the row pair (k1, 768 - k1) + real-FFT untangle +
//         mean-padding correction + |X|^2 / N, written slab-major
//         (PS[k1 + 768 m] at float m of row k1's own, already consumed, storage);
// pass T: slab-major -> natural bin order for the harmonic sum.
// Against the three-pass transform (fft_passes.hip) the 50 MB complex
// intermediate crosses the memory hierarchy twice instead of four times.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "fft_kernels.hpp"

namespace brp {
namespace hipk {

constexpr uint32_t kFft2L1 = 768;                 // column length (3 * 16 * 16, rows >= 256 are padding)
constexpr uint32_t kFft2R = 8192;                 // row length (2 * 16 * 16 * 16)
constexpr uint32_t kFft2M = kFft2L1 * kFft2R;     // 6 291 456
constexpr uint32_t kFft2ColsA = 16;               // pass-A columns per workgroup (128-B row segments)
constexpr uint32_t kFft2PartialsA = kFft2R / kFft2ColsA;  // pass-A workgroups (= partial sums) per template

// The plan applies when M matches and every sample lies in rows n1 < 256
// (2 * 256 * R = 2^22 >= n_unpadded >= n_steps).
inline bool fft2_supported(uint32_t M, uint32_t n_unpadded) {
  return M == kFft2M && n_unpadded <= 2u * 256u * kFft2R;
}

struct ColAArgs {
  float2* out;                 // [batch][M]
  const float* series;         // [slots][n_unpadded]
  uint32_t n_unpadded;
  const TemplateDev* tmpl;     // [batch]
  double* partials;            // [batch][kFft2PartialsA] sums of (sample - mu0)
  TwiddleTable tw;             // W_4M^e (period 2N)
  const float2* w768;          // W_768^e, e < 768
  uint32_t* reset;             // zeroed by workgroup (0, 0) when non-null (the batch's candidate counter)
};

struct RowBArgs {
  float2* buf;                 // [batch][M]: pass-A rows in, slab-major spectrum out
  TwiddleTable tw;
  const float2* w512;          // W_512^e, e < 512
  const float2* w8k;           // W_8192^e, e < 8192
  uint32_t limit;              // bins k < limit only
  float norm;                  // 1/N
  const TemplateDev* tmpl;     // n_steps
  const double* partials;      // pass-A sums, reduced in a fixed order by every workgroup
  // Nyquist bin M (natural order, when M < limit)
  float* ps;
  _Float16* ps16;
  uint32_t ps_stride;
};

struct PsTArgs {
  const float2* buf;           // slab-major spectrum (pass B)
  float* ps;                   // natural order [batch][ps_stride] (or ps16)
  _Float16* ps16;
  uint32_t ps_stride;
  uint32_t limit;
};

hipError_t launch_colA(const ColAArgs& a, int batch, hipStream_t s);
hipError_t launch_rowB(const RowBArgs& a, int batch, hipStream_t s);
hipError_t launch_psT(const PsTArgs& a, int batch, hipStream_t s);

}  // namespace hipk
}  // namespace brp
