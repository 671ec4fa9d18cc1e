// Chirp-z (Bluestein) transform for FFT lengths the three-pass kernels do not
// factor (implementation: bluestein.hip).
//
// The reference accepts any padding -P in [1, 10] and forms
// nsamples = (int)(P * N_u + 0.5) (demod_binary.c:226-244, 782); FFTW and cuFFT
// plan any length (demod_binary_fft_fftw.c:70, cuda/app/demod_binary_cuda.cu:862).
// Here a length-Mb DFT (Mb = N/2 of the packed real transform for even N, N
// itself for odd N) is
//   A_k = w_k * sum_n (a_n w_n) conj(w_{k-n}),   w_n = exp(-pi i n^2 / Mb),
// a circular convolution of length L >= 2 Mb - 1 computed with two length-L
// transforms of the smooth three-pass FFT:
//   y = chirp(a) (zero padded)          bs_chirp_in_kernel (templates: pass 1, P1_CHIRP*)
//   FFT_L(y) * H -> conj                 pass 1, 2, pass3_cplx (C3_MULCONJ)
//   FFT_L again -> conj * w / L          pass 1, 2, pass3_cplx (C3_CHIRP)
// with H = FFT_L(conj chirp, wrapped) precomputed once per plan. The template
// transforms run the convolution in transposed form instead: the DFT matrix
// is symmetric, so the inverse's three passes can run in reverse order on the
// forward transform's row layout --
//   pass 1 (P1_CHIRP*), pass 2           forward, rows (k1, k2) over n3 left in place
//   pass3_mid                            row FFT, * H (row layout), conj, row FFT, twiddle
//   pass 2 (rev), pass 1 (P1_REV_CHIRP)  columns over k2, then k1; conj * w / L, n < Mb
// -- five passes instead of six, and no natural-order (64-B piece) stores of
// the spectrum in between (round 5, profiles/README.md). The consumers
// (power spectrum with the mean-padding correction, whitening spectrum, real
// output of the inverse) are the bs_*_kernel launchers below.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "fft_kernels.hpp"
#include "hip_common.hpp"

namespace brp {
namespace hipk {

// (templates never materialise their chirp-multiplied input: pass 1 computes
// it from the series, Pass1Mode P1_CHIRP2 / P1_CHIRP1)
enum BsInMode : int {
  BS_IN_REAL2 = 2,      // whitening forward, even N: zero-padded real series pairs
  BS_IN_REAL1 = 3,      // whitening forward, odd N
  BS_IN_CONJ = 4,       // whitening inverse, even N: conj(z[n]) of the tangled half spectrum
  BS_IN_HERM_CONJ = 5,  // whitening inverse, odd N: conj of the Hermitian extension of spec
  BS_IN_HCHIRP = 6,     // setup: the wrapped conjugate chirp (input of H = FFT_L(h))
};

struct BsInArgs {
  float2* y;                   // [batch][L] chirp-multiplied, zero-padded input
  uint32_t L, Mb;              // convolution length, DFT length
  uint32_t nsamples;           // N
  TwiddleTable chirp;          // W_{2 Mb}
  // whitening
  const float* real_in;        // BS_IN_REAL*: n_real samples, zero beyond
  uint32_t n_real;
  const float2* cplx_in;       // BS_IN_CONJ: z[Mb]; BS_IN_HERM_CONJ: spec[fft_size]
  uint32_t w2, fft_size;       // BS_IN_HERM_CONJ: bins q < w2 or >= fft_size - w2 count as zero
};

enum Pass3CplxMode : int {
  C3_PLAIN = 0,    // natural-order complex output
  C3_MULCONJ = 1,  // conj(Z_n * H_n)
  C3_CHIRP = 2,    // conj(Z_n) * w_n * scale for n < n_out
};

struct Pass3CplxArgs {
  const float2* buf;           // [batch][M] after passes 1 and 2
  uint32_t L1, L2, L3, C, M;
  FFTTables tb;
  float2* out;                 // [batch][out_stride]
  size_t out_stride;
  const float2* h;             // C3_MULCONJ: H [M]
  TwiddleTable chirp;          // C3_CHIRP
  uint32_t n_out;
  float scale;
};

// template power spectrum from A (the DFT of length Mb), with the analytic
// mean-padding correction and 1/N normalisation; writes bins k < limit
struct BsPowerArgs {
  const float2* A;             // [batch][L]
  uint32_t L, Mb, nsamples;
  TwiddleTable tw;             // W_2N
  uint32_t limit;
  float* ps;                   // [batch][ps_stride]
  _Float16* ps16;              // fp16 spectrum instead (config 5) when non-null
  uint32_t ps_stride;
  float norm;                  // 1/N
  const TemplateDev* tmpl;
  const double* delta;         // [batch] mean of the centred samples (pass 2 of the first FFT)
  // paired odd-N transforms (P1_CHIRP1_PAIR): transform p holds templates 2p
  // (real part) and 2p + 1 (imaginary part, < n_tmpl); A is [transform][L]
  bool pair;
  uint32_t n_tmpl;
};

hipError_t launch_bs_chirp_in(BsInMode mode, const BsInArgs& a, int batch, uint32_t* n_partials, hipStream_t s);
uint32_t bs_chirp_in_blocks(uint32_t L);
hipError_t launch_pass3_cplx(const FFTPlan3& plan, Pass3CplxMode mode, const Pass3CplxArgs& a, int batch,
                             hipStream_t s);
hipError_t launch_bs_power(const BsPowerArgs& a, int batch, hipStream_t s);
// H (natural order) -> the row layout of the transposed convolution (pass3_mid)
hipError_t launch_bs_rows(const float2* H, float2* hp, uint32_t L1, uint32_t L2, uint32_t L3, hipStream_t s);
// whitening: A -> complex half spectrum X_k, k < fft_size (unnormalised)
hipError_t launch_bs_spec(const float2* A, uint32_t Mb, uint32_t nsamples, const TwiddleTable& tw, uint32_t fft_size,
                          float2* spec, hipStream_t s);
// whitening inverse: A -> n_out real samples times scale
hipError_t launch_bs_real_out(const float2* A, uint32_t Mb, uint32_t nsamples, float scale, float* out,
                              uint32_t n_out, hipStream_t s);

}  // namespace hipk
}  // namespace brp
