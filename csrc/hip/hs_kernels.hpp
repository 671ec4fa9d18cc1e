// Harmonic summing + threshold compaction (implementation: harmonic_sum.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace brp {
namespace hipk {

// Fundamental-level bins i per workgroup: the tile plus its 4-bin halo fill
// 4 x 256 lanes exactly (1024 would leave a fifth pass of 4 lanes; +1.4 %).
constexpr int kHsTile = 1008;

enum HSMode : int {
  HS_F32 = 0,  // gathers from the fp32 spectrum (exact)
  HS_F16 = 1,  // gathers from the fp16 spectrum (config 5)
};

struct HSArgs {
  int mode;               // HSMode
  const float* ps;        // [batch][ps_stride] fp32 spectrum (HS_F32)
  const _Float16* ps16;   // [batch][ps_stride] fp16 spectrum (HS_F16)
  uint32_t ps_stride;
  uint32_t w2, fhi, hhi;  // window_2, fundamental_idx_hi, harmonic_idx_hi
  int32_t i_start;        // first i of tile 0 (== 8 mod 16, <= w2; -8 for windows below 16)
  const float* thr;       // [batch][kHsThrStride] device thresholds per template
  // one compact list per batch: list[0].x = number of entries (atomic; may
  // exceed cap), list[1 + q] = (hs_pack(template, level, bin), power bits)
  uint2* list;
  uint32_t cap;
  // pruned path (HS_F32): maxima of the spectrum over cells of 2^cell_shift
  // bins (2 or 3), [batch][pyr_stride]
  bool prune;
  int cell_shift;
  bool direct;  // bounds read straight from global memory (no LDS staging; 8-bin cells)
  bool xcd;     // pruned kernel: contiguous block ranges per XCD (BRP_HS_XCD=1, experiment)
  float* pyr;
  uint32_t pyr_stride;
  uint32_t key_base;  // index of template 0 of this launch within the batch's candidate list
};

// cells covering the spectrum row, room for 4-bin cells (bins >= hhi count as 0)
__host__ __device__ constexpr uint32_t hs_pyr_stride(uint32_t ps_stride) { return ps_stride / 4 + 8; }
// 16-bin blocks of the pruned path (tile grid of kHsTile, i_start == 8 mod 16)
uint32_t hs_num_blocks(int32_t i_start, uint32_t hhi);

constexpr uint32_t kHsThrStride = 8;  // floats per template in the threshold array (5 used)
constexpr uint32_t kHsBinBits = 23;  // bins < 2^23, levels < 8, templates per batch < 64
constexpr uint32_t kHsMaxBatch = 64;
__host__ __device__ constexpr uint32_t hs_pack(uint32_t k, uint32_t h, uint32_t bin) {
  return (k << 26) | (h << kHsBinBits) | bin;
}

uint32_t hs_num_tiles(int32_t i_start, uint32_t hhi);
hipError_t launch_harmonic_sum(const HSArgs& a, int batch, hipStream_t s);

}  // namespace hipk
}  // namespace brp
