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
  // 8-bin cells of the bins with residue mod row_c below row_c / 2 already
  // written (pass 3 fused them, rows of row_c bins, row_l rows up to M): the
  // cell kernel computes only the others (mirror half and past M)
  bool cells_ready;
  uint32_t row_c, row_l;
  uint32_t cells_cpt;  // fp32 8-bin cells per thread of the cell kernel (1: hs_cells_kernel, 4: hs_cells8_kernel<4>)
  uint32_t key_base;  // index of template 0 of this launch within the batch's candidate list
  uint32_t bin_bits;  // candidate key layout (hs_pack): bins < 2^bin_bits
  float* dense;       // select path: [batch][5][dense_stride] level values (HsSelectArgs)
  uint32_t dense_stride;
};

// cells covering the spectrum row, room for 4-bin cells (bins >= hhi count as 0)
__host__ __device__ constexpr uint32_t hs_pyr_stride(uint32_t ps_stride) { return ps_stride / 4 + 8; }
// 16-bin blocks of the pruned path (tile grid of kHsTile, i_start == 8 mod 16)
uint32_t hs_num_blocks(int32_t i_start, uint32_t hhi);

constexpr uint32_t kHsThrStride = 8;  // floats per template in the threshold array (5 used)
constexpr uint32_t kHsMaxBatch = 64;  // templates per submitted batch (threshold / parameter area)
// Candidate key: template index in the batch | level (3 bits) | bin (bin_bits),
// with bin_bits sized to the geometry's fundamental_idx_hi (hs_bin_bits), so any
// -f / -P the reference accepts fits (fundamental_idx_hi <= fft_size ~ 2.1e7 on a
// 2^22-sample WU at -P 10: 25 bits, 4 template bits). Beyond 2^29 bins no key fits.
constexpr uint32_t kHsMaxBinBits = 29;
__host__ __device__ constexpr uint32_t hs_pack(uint32_t k, uint32_t h, uint32_t bin, uint32_t bin_bits) {
  return static_cast<uint32_t>(static_cast<uint64_t>(k) << (bin_bits + 3)) | (h << bin_bits) | bin;
}
inline uint32_t hs_bin_bits(uint32_t fhi) {
  uint32_t b = 1;
  while (b < 32 && (1ull << b) < fhi) ++b;  // every bin < fhi <= 2^b
  return b;
}
// templates a batch's keys can address (0: the geometry has no key layout)
inline uint32_t hs_key_templates(uint32_t bin_bits) {
  if (bin_bits > kHsMaxBinBits) return 0;
  const uint64_t n = 1ull << (32 - 3 - bin_bits);
  return static_cast<uint32_t>(n < kHsMaxBatch ? n : kHsMaxBatch);
}

uint32_t hs_num_tiles(int32_t i_start, uint32_t hhi);
hipError_t launch_harmonic_sum(const HSArgs& a, int batch, hipStream_t s);

// ---- bounded candidate output (the overflow path)
// For every template and level, a bin whose level value has >= K values of
// the same template and level strictly above it can never enter the K-entry
// table level (its K betters are distinct bins that the
// table then holds at >= their powers), so emitting only the values >= the
// K-th largest (ties kept) gives the in-order applier exactly the table of
// the full list. Used when a batch's list overflows (no -W: raw powers put
// nearly every bin above the chi^2 thresholds): the level values are written
// densely, the K-th largest found by a 3-round radix select on their bits
// (positive floats order like their bit patterns), and only those emitted.
struct HsSelectArgs {
  float* dense;           // [batch][5][dense_stride]: level value if > threshold, else 0
  uint32_t dense_stride;  // >= fhi
  uint32_t* hist;         // [batch][5][kHsSelBins] radix histograms
  uint32_t* state;        // [batch][5][4]: prefix, k remaining, fewer-than-K flag, positives
  uint32_t k;             // values kept per template and level (kCandPerLevel)
};
constexpr uint32_t kHsSelBins = 2048;
// list[0].y accumulates the number of values above threshold of the batch
// (what the compacting path would have emitted; the engine's mode switch)
hipError_t launch_harmonic_sum_select(const HSArgs& a, const HsSelectArgs& s, int batch, hipStream_t st);

}  // namespace hipk
}  // namespace brp
