// Shared device-side helpers for the MI355X (gfx950) kernels.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#include "../core/errors.hpp"
#include "../core/log.hpp"
#include "checked.hpp"

namespace brp {
namespace hipk {

#define BRP_HIP_CHECK(expr, code)                                                                  \
  do {                                                                                             \
    hipError_t _e = (expr);                                                                        \
    if (_e != hipSuccess) {                                                                        \
      ::brp::log_message(::brp::LOG_ERROR, true, "HIP error %s at %s:%d: %s\n", hipGetErrorName(_e), \
                         __FILE__, __LINE__, #expr);                                               \
      return (code);                                                                               \
    }                                                                                              \
  } while (0)

constexpr int kWave = 64;

// Two-level table for W_{2N}^j = exp(-i pi j / N), j in [0, 2N):
//   W^j = hi[j >> kTwLoBits] * lo[j & (2^kTwLoBits - 1)]
// Both tables are tiny (L1/L2 resident); the product is accurate to ~1e-7.
constexpr int kTwLoBits = 12;
struct TwiddleTable {
  const float2* hi;
  const float2* lo;
  uint64_t period;  // 2N
  // 1 / period (tw_lookup's reduction by a double-precision reciprocal; 0:
  // the plain 64-bit modulo). Set by the host for every table (periods < 2^32).
  double inv_period = 0.0;
};

#if defined(__HIP__)
// Complex arithmetic as packed-FP32 vector operations (v_pk_add_f32,
// v_pk_mul_f32, v_pk_fma_f32). Written on a native 2-float vector, the
// element broadcasts, swaps and sign changes fold into the instructions'
// op_sel / neg modifiers or into a scalar-register sign pair; written per
// component (make_float2(a.x * b.x - a.y * b.y, ...)) the compiler paired
// the operands with register moves and sign flips with v_xor: a complex
// product took ~4.5 VALU instead of 2, a radix-4 butterfly ~1.5x its packed
// count (tools/isa_mix.py, round 5).
using f2v = float __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2v vec(float2 a) { return f2v{a.x, a.y}; }
__device__ __forceinline__ float2 unvec(f2v a) { return make_float2(a.x, a.y); }
// a * b: a.x * (b.x, b.y) + a.y * (-b.y, b.x), one v_pk_mul_f32 + one v_pk_fma_f32.
// The fma is explicit and keeps the a.y products exact: contracted the other
// way (a.x products exact, the compiler's choice for the plain expression) the
// chirp-z spectrum of plan 240 x 240 x 256 drew 4x the worst-bin error (3.9e-4
// against 9.3e-5 of the component form, tools/chirp_err.py, round 5)
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  const f2v av = vec(a), bv = vec(b);
  const f2v bs = {-bv.y, bv.x};
  return unvec(__builtin_elementwise_fma(av.yy, bs, av.xx * bv));
}
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return unvec(vec(a) + vec(b)); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return unvec(vec(a) - vec(b)); }
__device__ __forceinline__ float2 conjf2(float2 a) { return make_float2(a.x, -a.y); }
// multiply by -i (forward-transform rotation)
__device__ __forceinline__ float2 mul_mi(float2 a) { return make_float2(a.y, -a.x); }
__device__ __forceinline__ float2 cscale(float2 a, float s) { return unvec(vec(a) * s); }
// a + s (-i) d = (a.x + s d.y, a.y - s d.x) and a - s (-i) d, one v_pk_fma_f32
// each (the swap in op_sel, the signs in a scalar pair; s = 1 is exact: one
// rounding, the same value as the add)
__device__ __forceinline__ float2 add_mi(float2 a, float2 d, float s = 1.0f) {
  const f2v sg = {s, -s};
  return unvec(__builtin_elementwise_fma(vec(d).yx, sg, vec(a)));
}
__device__ __forceinline__ float2 sub_mi(float2 a, float2 d, float s = 1.0f) {
  const f2v sg = {-s, s};
  return unvec(__builtin_elementwise_fma(vec(d).yx, sg, vec(a)));
}
// a + s b (one v_pk_fma_f32)
__device__ __forceinline__ float2 cfma(float s, float2 b, float2 a) {
  return unvec(__builtin_elementwise_fma(f2v{s, s}, vec(b), vec(a)));
}

// j mod m (m < 2^32, j < 2^60) from a double-precision quotient estimate,
// corrected exactly: gfx950 has no 64-bit integer divide, and the compiler's
// 64-bit urem is a ~100-instruction sequence per call -- measured as most of
// the chirp-z kernels' arithmetic (n^2 mod 2 Mb per element, round 5). The
// estimate q is within a few units of j / m (one rounding of j and of the
// product), so the two loops run at most a couple of times.
__device__ __forceinline__ uint32_t mod_u64(uint64_t j, uint32_t m, double inv_m) {
  const uint64_t q = static_cast<uint64_t>(static_cast<double>(j) * inv_m);
  int64_t r = static_cast<int64_t>(j - q * m);
  while (r < 0) r += m;
  while (r >= static_cast<int64_t>(m)) r -= m;
  return static_cast<uint32_t>(r);
}

__device__ __forceinline__ float2 tw_lookup(const TwiddleTable& t, uint64_t j) {
  if (t.inv_period != 0.0 && j < (1ull << 60)) j = mod_u64(j, static_cast<uint32_t>(t.period), t.inv_period);
  else j %= t.period;
  const float2 a = BRP_LD(&t.hi[j >> kTwLoBits]);
  const float2 b = BRP_LD(&t.lo[j & ((1u << kTwLoBits) - 1)]);
  return cmul(a, b);
}
// same for an exponent already known to be < period (32-bit fast path)
__device__ __forceinline__ float2 tw_lookup32(const TwiddleTable& t, uint32_t j) {
  const float2 a = BRP_LD(&t.hi[j >> kTwLoBits]);
  const float2 b = BRP_LD(&t.lo[j & ((1u << kTwLoBits) - 1)]);
  return cmul(a, b);
}

// XCD-aware workgroup order: the dispatcher deals workgroups round-robin over
// the 8 XCDs (b, b+8, ... share one XCD and its L2). Remap so that each XCD
// gets a contiguous range of logical workgroups (bijective for any nwg).
// Placement is a speed hint only; correctness never depends on it.
__device__ __forceinline__ uint32_t xcd_remap(uint32_t bid, uint32_t nwg) {
  constexpr uint32_t kXcd = 8;
  const uint32_t q = nwg / kXcd, r = nwg % kXcd, x = bid % kXcd, k = bid / kXcd;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + k;
}

// maximum over the wave's active lanes of a value below 2^BITS, uniform
// result: one ballot per bit from the top. A partial last wave (workgroups of
// 48 / 80 / 112 threads) has inactive lanes, and a cross-lane shuffle would
// read their stale registers; a ballot only counts lanes that run.
template <int BITS>
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
  static_assert(BITS >= 1 && BITS <= 32, "value bits");
  uint32_t m = 0;
#pragma unroll
  for (int bit = BITS - 1; bit >= 0; --bit) {
    const uint32_t c = m | (1u << bit);
    if (__ballot(v >= c) != 0) m = c;
  }
  return __builtin_amdgcn_readfirstlane(m);
}

// wave-level sum (64 lanes) of a double
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}
#endif  // __HIP__

}  // namespace hipk
}  // namespace brp
