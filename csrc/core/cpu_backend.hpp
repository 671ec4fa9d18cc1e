// CPU golden backend: the executable specification of the per-template
// pipeline (reference CPU backend: demod_binary_resamp_cpu.c, demod_binary_fft_fftw.c,
// hs_common.c) and of the whitening/zapping step (demod_binary.c:857-1079).
// The HIP backend is validated against these functions.
#pragma once

#include <cstdint>
#include <vector>

#include "io.hpp"
#include "resamp_math.hpp"
#include "search_core.hpp"

namespace brp {

// Resample `series` (n_unpadded samples) into `out` (nsamples): nearest
// neighbour gather for i < n_steps, mean padding afterwards.
void cpu_resample(const float* series, const ResampParams& p, std::vector<float>& out, uint32_t* n_steps_out,
                  float* mean_out);

// Normalised power spectrum ps[k] = |X_k|^2 / N for k < fft_size, ps[0] = 0
// (double precision FFT).
void cpu_power_spectrum(const std::vector<float>& x, uint32_t fft_size, std::vector<float>& ps);

// Harmonic summing with the exact reference index arithmetic and float
// summation order (hs_common.c:33-171). Returns, per level h, the bins
// j in [window_2, fundamental_idx_hi) whose summed power exceeds thr[h]
// (ascending). If sumspec != nullptr it receives the full max-power arrays
// (5 x fundamental_idx_hi, level 0 = ps).
void cpu_harmonic_sum(const std::vector<float>& ps, const SearchGeometry& g, const float thr[kNumHarmonicLevels],
                      std::vector<BinPower> out[kNumHarmonicLevels], std::vector<float>* sumspec = nullptr);

// Whitening + RFI zapping of the time series in place.
int cpu_whiten(std::vector<float>& series, const SearchGeometry& g, const SearchOptions& opt,
               const std::vector<ZapRange>& zaps);

// Deterministic RFI noise for zapping: for every zap range, every bin
// idx_min..idx_max (inclusive) gets (re, im) Gaussian noise drawn in the
// reference order. Shared by CPU and HIP whitening.
struct ZapNoise {
  std::vector<uint32_t> bin;
  std::vector<float> re, im;
};
void make_zap_noise(int32_t seed, const SearchGeometry& g, const SearchOptions& opt,
                    const std::vector<ZapRange>& zaps, ZapNoise& noise);

}  // namespace brp
