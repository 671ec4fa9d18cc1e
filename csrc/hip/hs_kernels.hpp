// Harmonic summing + threshold compaction (implementation: harmonic_sum.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace brp {
namespace hipk {

constexpr int kHsTile = 1024;  // fundamental-level bins i per workgroup

enum HSVariant : int {
  HS_GATHER = 0,            // one lane per i, 16 gathers (tiles + halo, LDS level maxima)
  HS_REGISTER_BLOCKED = 1,  // one lane per 16 i, 16 contiguous runs per lane (fp32 spectrum)
  HS_QUAD = 2,              // one lane per 4 i, one 16-byte load per harmonic (fp32 spectrum)
};

struct HSArgs {
  int variant;            // HSVariant
  int rb_occupancy;       // register-blocked kernel: minimum waves per SIMD the compiler targets (0 = free)
  const float* ps;        // [batch][ps_stride]
  const _Float16* ps16;   // fp16 spectrum (config 5) instead of `ps` when non-null
  uint32_t ps_stride;
  uint32_t w2, fhi, hhi;  // window_2, fundamental_idx_hi, harmonic_idx_hi
  uint32_t i_start;       // first i of tile 0 (== 8 mod 16, <= w2)
  const float* thr;       // [batch][kHsThrStride] device thresholds per template
  // one compact list per batch: list[0].x = number of entries (atomic; may
  // exceed cap), list[1 + q] = (hs_pack(template, level, bin), power bits)
  uint2* list;
  uint32_t cap;
  int staged_harmonics;   // harmonics 1..n staged in LDS (0, 4, 8 or 16), the rest gathered per i
  uint32_t tile;          // bins i per workgroup (0 = kHsTile; 496, 1008, 2032 without staging)
  uint32_t xcd;           // nonzero: consecutive tiles on one XCD (shared harmonic lines stay in its L2)
};

constexpr uint32_t kHsThrStride = 8;  // floats per template in the threshold array (5 used)
constexpr uint32_t kHsBinBits = 23;  // bins < 2^23, levels < 8, templates per batch < 64
constexpr uint32_t kHsMaxBatch = 64;
__host__ __device__ constexpr uint32_t hs_pack(uint32_t k, uint32_t h, uint32_t bin) {
  return (k << 26) | (h << kHsBinBits) | bin;
}

uint32_t hs_num_tiles(uint32_t i_start, uint32_t hhi, uint32_t tile = kHsTile);
uint32_t hs_rb_num_groups(uint32_t w2, uint32_t hhi);
hipError_t launch_harmonic_sum(const HSArgs& a, int batch, hipStream_t s);

}  // namespace hipk
}  // namespace brp
