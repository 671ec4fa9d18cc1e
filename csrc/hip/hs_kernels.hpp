// Harmonic summing + threshold compaction (implementation: harmonic_sum.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace brp {
namespace hipk {

constexpr int kHsTile = 1024;  // fundamental-level bins i per workgroup

struct HSArgs {
  const float* ps;        // [batch][ps_stride]
  uint32_t ps_stride;
  uint32_t w2, fhi, hhi;  // window_2, fundamental_idx_hi, harmonic_idx_hi
  uint32_t i_start;       // first i of tile 0 (== 8 mod 16, <= w2)
  const float* thr;       // [5] device thresholds for the whole batch
  uint32_t* counts;       // [batch][5] (atomic; may exceed cap)
  uint2* cands;           // [batch][5][cap]: (bin, power bits)
  uint32_t cap;
};

uint32_t hs_num_tiles(uint32_t i_start, uint32_t hhi);
hipError_t launch_harmonic_sum(const HSArgs& a, int batch, hipStream_t s);

}  // namespace hipk
}  // namespace brp
