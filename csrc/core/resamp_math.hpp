// Scalar math of the time-domain resampling, shared by the CPU golden model and
// the HIP kernels so that both pick exactly the same nearest-neighbour sample.
//
// Semantics follow the reference CPU backend (demod_binary_resamp_cpu.c:80-136 and
// sincosLUTLookup, erp_utilities.cpp:176-209): float arithmetic evaluated left
// to right with NO fused multiply-add (the CUDA port forbids contraction with
// __fmul_rn/__fadd_rn for the same reason, cuda/app/demod_binary_cuda.cuh:40-80).
#pragma once

#include <cmath>
#include <cstdint>

#include "sincos_lut.hpp"

#if defined(__HIPCC__) || defined(__HIP__)
#define BRP_HD __host__ __device__
#else
#define BRP_HD
#endif

namespace brp {

// Per-template resampling parameters (reference RESAMP_PARAMS, structs.h:151-161).
struct ResampParams {
  uint32_t nsamples;           // padded length N
  uint32_t nsamples_unpadded;  // N_u
  uint32_t fft_size;           // N/2 + 1
  float tau;                   // projected orbital radius [s]
  float Omega;                 // 2 pi / P_orb [rad/s]
  float Psi0;                  // initial orbital phase [rad]
  float dt;                    // sample time [s]
  float step_inv;              // 1/dt
  float S0;                    // tau*sin(Psi0)/dt
};

// sin(x) from the 64-sample LUT with a 2nd-order Taylor correction.
BRP_HD inline float lut_sin(float x, const float* __restrict__ sin_lut,
                            const float* __restrict__ cos_lut) {
#pragma clang fp contract(off)
  float ipart;
  float xt = modff(kLutTwoPiInv * x, &ipart);
  if (xt < 0.0f) xt += 1.0f;
  const int i0 = static_cast<int>(xt * kLutResF + 0.5f);
  const float d = kLutTwoPi * (xt - kLutResFInv * static_cast<float>(i0));
  const float d2 = d * (0.5f * d);
  const float ts = sin_lut[i0];
  const float tc = cos_lut[i0];
  return (ts + d * tc) - d2 * ts;
}

// del_t[i]: arrival-time offset of pulsar-frame sample i, in samples.
BRP_HD inline float resamp_del_t(uint32_t i, const ResampParams& p,
                                 const float* __restrict__ sin_lut,
                                 const float* __restrict__ cos_lut) {
#pragma clang fp contract(off)
  const float t = static_cast<float>(i) * p.dt;
  const float s = lut_sin(p.Omega * t + p.Psi0, sin_lut, cos_lut);
  return p.tau * s * p.step_inv - p.S0;
}

// Detector-frame sample that pulsar-frame sample i maps to (nearest neighbour).
// The +0.5 is a double constant in the reference, so the add is done in double.
BRP_HD inline int resamp_nearest(uint32_t i, float del_t) {
#pragma clang fp contract(off)
  const float x = static_cast<float>(i) - del_t;
  return static_cast<int>(static_cast<double>(x) + 0.5);
}

// Same result as resamp_nearest without double arithmetic, valid for
// |x| < 2^23: there float(x) + 0.5f is exact (ulp(x) <= 0.5), so both round
// trips truncate the same value. Callers guarantee i < n_unpadded <= 2^23.
BRP_HD inline int resamp_nearest_f(uint32_t i, float del_t) {
#pragma clang fp contract(off)
  const float x = static_cast<float>(i) - del_t;
  return static_cast<int>(x + 0.5f);
}

// True if sample m must be dropped at the end of the series
// (reference loop `while(n_steps - del_t[n_steps] >= N_u - 1) n_steps--`).
BRP_HD inline bool resamp_beyond_end(uint32_t m, float del_t, uint32_t n_unpadded) {
#pragma clang fp contract(off)
  return static_cast<float>(m) - del_t >= static_cast<float>(n_unpadded - 1);
}

// Number of resampled samples taken from the series (the rest is padding):
// the reference scans down from N_u - 1 while the sample maps beyond the end
// (demod_binary_resamp_cpu.c:94-99). m - del_t(m) rises monotonically
// (|tau * Omega| << 1), so the crossing is bracketed by doubling steps and
// bisection, and the reference's descending scan is replayed from 64 samples
// above it: same result, ~30 instead of up to ~5000 LUT evaluations.
inline uint32_t resamp_n_steps(const ResampParams& p, const float* sin_lut, const float* cos_lut) {
  const uint32_t nu = p.nsamples_unpadded;
  auto beyond = [&](uint32_t m) { return resamp_beyond_end(m, resamp_del_t(m, p, sin_lut, cos_lut), nu); };
  uint32_t hi = nu - 1;
  if (!beyond(hi)) return hi;
  uint32_t lo = hi, span = 64;
  for (;;) {
    lo = hi > span ? hi - span : 0;
    if (lo == 0 || !beyond(lo)) break;
    hi = lo;
    span *= 2;
  }
  while (hi - lo > 1) {
    const uint32_t mid = lo + (hi - lo) / 2;
    if (beyond(mid)) hi = mid;
    else lo = mid;
  }
  uint32_t n = lo + 64 < nu - 1 ? lo + 64 : nu - 1;
  while (n > 0 && beyond(n)) n--;
  return n;
}

// The reference's plain descending scan (test oracle for resamp_n_steps).
inline uint32_t resamp_n_steps_scan(const ResampParams& p, const float* sin_lut, const float* cos_lut) {
  const uint32_t nu = p.nsamples_unpadded;
  uint32_t n = nu - 1;
  while (n > 0 && resamp_beyond_end(n, resamp_del_t(n, p, sin_lut, cos_lut), nu)) n--;
  return n;
}

// Host-side derivation of the per-template parameters from one template-bank
// line (demod_binary.c:1207-1238). Note the reference is compiled as C++, so
// sin(float) resolves to the float overload.
inline ResampParams make_resamp_params(uint32_t nsamples, uint32_t n_unpadded, uint32_t fft_size,
                                       float dt, float step_inv, float P, float tau,
                                       float Psi0) {
#pragma clang fp contract(off)
  ResampParams r;
  r.nsamples = nsamples;
  r.nsamples_unpadded = n_unpadded;
  r.fft_size = fft_size;
  r.tau = tau;
  r.Omega = static_cast<float>(2.0 * M_PI / static_cast<double>(P));
  r.Psi0 = Psi0;
  r.dt = dt;
  r.step_inv = step_inv;
  r.S0 = tau * std::sin(Psi0) * step_inv;
  return r;
}

}  // namespace brp
