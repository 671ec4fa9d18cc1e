// Kernel argument blocks and launchers of the three FFT passes
// (implementation: fft_passes.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "../core/resamp_math.hpp"
#include "fft_plan.hpp"
#include "hip_common.hpp"

namespace brp {
namespace hipk {

// Per-template device parameters (one entry per template of a batch).
struct TemplateDev {
  ResampParams p;
  uint32_t n_steps;   // samples taken from the series (rest is mean padding)
  float mu0;          // reference level subtracted before the FFT
  uint32_t wu;        // work-unit slot: series = Pass1Args::series + wu * n_unpadded
  uint32_t pad;
};

// Twiddle tables precomputed on the host per FFT plan (single rounding from
// double precision; loaded contiguously by the kernels instead of being
// assembled per element).
struct FFTTables {
  const float2* st1;    // stage table W_L1^e, padded order e + e/16
  const float2* st2;    // stage table W_L2^e
  const float2* st3;    // stage table W_L3^e
  const float2* p1;     // [L2][L1]  W_{L1 L2}^{n2 k1}
  const float2* p2col;  // [L1][L3]  W_M^{n3 k1}
  const float2* p2lo;   // [256]     W_{L2 L3}^{i}
  const float2* p2hi;   // [<=1024]  W_{L2 L3}^{256 i}
  const float2* p3;     // [4 L3]    W_2N^{C i}
};

enum Pass1Mode : int {
  P1_RESAMPLE = 0,   // fused nearest-neighbour resampling of the time series
  P1_REAL = 1,       // zero-padded real series
  P1_COMPLEX_CONJ = 2,  // complex input, conjugated (inverse transform)
  P1_COMPLEX = 3,       // complex input as is (chirp-z convolutions, bluestein_kernels.hpp)
  // chirp-z template transforms (bluestein_kernels.hpp): the resampled,
  // centred series times the chirp w_n for n < Mb, zero beyond, straight from
  // the series (the chirp-multiplied input is never materialised)
  P1_CHIRP2 = 4,        // even N: (x[2n], x[2n+1]) w_n
  P1_CHIRP1 = 5,        // odd N: x[n] w_n
  // odd N, two templates per transform: (x_a[n] + i x_b[n]) w_n for templates
  // 2p and 2p + 1 of the launch (X_a, X_b separate by conjugate symmetry in
  // bs_power_kernel): half the chirp-z work per template
  P1_CHIRP1_PAIR = 6,
  // last pass of a chirp-z convolution's inverse transform in transposed
  // order (bluestein_kernels.hpp): columns over k1 of `cplx_in` (pass 2's
  // reverse output) -> natural-order n, then conj(.) * w_n * scale for n < Mb
  // into `out` (the length-Mb DFT A); no output twiddle
  P1_REV_CHIRP = 7,
};

struct Pass1Args {
  float2* out;                 // [batch][M]
  uint32_t L2L3, L3;
  TwiddleTable tw;
  FFTTables tb;
  // P1_RESAMPLE
  const float* series;         // [slots][n_unpadded] samples (slot per template: TemplateDev::wu)
  uint32_t n_unpadded;
  const TemplateDev* tmpl;     // [batch]
  double* partials;            // [batch][wg1] sums of (sample - mu0)
  uint32_t* reset;             // zeroed by workgroup (0, 0) when non-null (the batch's candidate counter)
  // P1_REAL
  const float* real_in;
  uint32_t n_real;
  // P1_COMPLEX_CONJ, P1_COMPLEX: [batch][M]
  const float2* cplx_in;
  // P1_CHIRP*: chirp W_{2 Mb}^{n^2} of the length-Mb DFT (also uses series/tmpl/partials)
  TwiddleTable chirp;
  uint32_t Mb;
  uint32_t n_tmpl;             // P1_CHIRP1_PAIR: templates of the launch (transform p: 2p, 2p + 1 < n_tmpl)
  float scale;                 // P1_REV_CHIRP: 1 / L
  bool lds_pass1;              // P1_RESAMPLE: LDS-staged pass1_kernel instead of pass1g_kernel (BRP_P1_LDS=1)
};

struct Pass2Args {
  float2* buf;                 // [batch][M], in place
  uint32_t L1, L2L3, L3;
  TwiddleTable tw;
  FFTTables tb;
  // mean-padding correction (template pipeline only, else nullptr): workgroup 0
  // of each template reduces pass 1's partial sums once, in a fixed order,
  // delta[b] = sum / n_steps
  const double* partials;      // [batch][n_partials]
  uint32_t n_partials;
  const TemplateDev* tmpl;
  double* delta;               // [batch]
  // templates per transform (2: paired chirp-z transforms, P1_CHIRP1_PAIR;
  // 0 counts as 1) and templates of the launch: transform p reduces the
  // partial sums of templates tpt p .. tpt p + tpt - 1 (< n_tmpl)
  uint32_t tpt, n_tmpl;
  // reverse (transposed) pass of a chirp-z convolution's inverse transform:
  // DFT over the column's k2 -> m2 with the output twiddle W_{L1 L2}^{k1 m2}
  // (p1 table) instead of pass 2's W_M^{n3 (k1 + L1 k2)}
  bool rev;
};

enum Pass3Mode : int {
  P3_POWER = 0,     // untangle + power spectrum (+ mean-padding correction)
  P3_COMPLEX = 1,   // untangle, complex half spectrum out (whitening)
  P3_POWER16 = 2,   // as P3_POWER, fp16 spectrum (Pass3Args::ps16; selected by launch_pass3)
};

struct Pass3Args {
  const float2* buf;           // [batch][M]
  uint32_t L1, L2, L3, C;      // C = L1*L2 rows
  uint32_t M;
  TwiddleTable tw;
  FFTTables tb;
  uint32_t limit;              // write bins k < limit only
  // P3_POWER
  float* ps;                   // [batch][ps_stride]
  _Float16* ps16;              // fp16 spectrum instead of `ps` when non-null
  uint32_t ps_stride;
  float norm;                  // 1/N (float)
  const TemplateDev* tmpl;     // n_steps per template
  const double* delta;         // [batch] mean-padding correction (pass 2)
  // P3_COMPLEX
  float2* spec;                // fft_size complex bins
  // P3_POWER with the pruned harmonic sum's 8-bin bound cells fused (when
  // non-null): cells[b * cells_stride + j] = max of bins 8j .. 8j + 7 (0 past
  // limit); the caller zeroes them first
  float* cells;
  uint32_t cells_stride, n_cells;
};

// Middle of a chirp-z convolution (bluestein_kernels.hpp), in place on the
// row layout pass 2 leaves: per row (k1, k2) the forward row FFT over n3 ->
// k3, times H in the same layout (hp[row][k3] = H[k1 + L1 k2 + L1 L2 k3]),
// conj, the row FFT of the transposed inverse transform (k3 -> m3) and its
// twiddle W_M^{m3 (k1 + L1 k2)}. Pass 2 (rev) and pass 1 (P1_REV_CHIRP) finish
// the inverse transform from there, so the convolution never writes the
// spectrum in natural order.
struct Pass3MidArgs {
  float2* buf;                 // [batch][M], in place
  const float2* hp;            // [M] H in row layout
  uint32_t L1, L2, L3;
  FFTTables tb;                // st3; p2col, p2lo, p2hi (the twiddle)
  bool whole_waves;            // 16 / 32 rows per workgroup where 8 rows are not whole waves (BRP_MID_WAVES=1, A/B)
};

// plain row pass of the inverse transform: conj, scale, write the first
// n_out real samples of the natural-order output
struct Pass3PlainArgs {
  const float2* buf;
  uint32_t L1, L2, L3, C;
  TwiddleTable tw;
  FFTTables tb;
  float scale;
  float* real_out;
  uint32_t n_out;              // real samples to write
};

hipError_t launch_pass1(const FFTPlan3& plan, Pass1Mode mode, const Pass1Args& a, int batch, hipStream_t s);
hipError_t launch_pass2(const FFTPlan3& plan, const Pass2Args& a, int batch, hipStream_t s);
hipError_t launch_pass3(const FFTPlan3& plan, Pass3Mode mode, const Pass3Args& a, int batch, hipStream_t s);
hipError_t launch_pass3_plain(const FFTPlan3& plan, const Pass3PlainArgs& a, hipStream_t s);
hipError_t launch_pass3_mid(const FFTPlan3& plan, const Pass3MidArgs& a, int batch, hipStream_t s);
// lengths of the transposed chirp-z convolution (pass3_mid, pass 2 rev, P1_REV_CHIRP)
bool chirp_rev_supported(const FFTPlan3& plan);

// code objects of the device modules onto the current device (each module's
// is otherwise loaded at its first launch); HipEngine::warm_up
hipError_t preload_fft_passes();
hipError_t preload_harmonic_sum();
hipError_t preload_whiten();
hipError_t preload_resample();
hipError_t preload_bluestein();
hipError_t preload_rmed_wide();

// lengths with compiled kernels
bool pass12_length_supported(uint32_t L);
bool pass3_length_supported(uint32_t L);

}  // namespace hipk
}  // namespace brp
