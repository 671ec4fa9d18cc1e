// Harmonic summing of 1/2/4/8/16 harmonics with on-device threshold compaction.
//
// For fundamental-level index i the summed power over 2^h harmonics is
//   S_h(i) = sum_{l=1}^{2^h} PS[(l*(16/2^h)*i + 8) >> 4]
// with the reference's exact integer rounding and float summation order
// (hs_common.c:33-171), and sumspec[h][j] = max S_h(i) over the 2^h
// consecutive i with round(i/2^h) == j.
//
// The CUDA port needs two kernels per template because its 16-thread tiling
// leaves 3 slots per 16 bins to a "gap" kernel
// (cuda/app/harmonic_summing_kernel.cuh:81-416). Here one workgroup owns every
// output group whose first i lies in its tile and computes a 4-sample halo, so
// one launch covers all levels. Instead of writing five dense sumspec arrays and
// dirty-page flags that the host then scans, each workgroup appends only the
// (bin, power) pairs above the device threshold to per-level candidate lists
// (wave-aggregated atomics); the host merges them into the candidate table.
#include <type_traits>
#include <utility>

#include "hip_common.hpp"
#include "hs_kernels.hpp"

namespace brp {
namespace hipk {

namespace {

constexpr int kThreads = 256;
constexpr int kHalo = 4;
__device__ __forceinline__ int sidx(int t) { return t + (t >> 4); }

__device__ __forceinline__ void emit(uint32_t* counter, uint2* list, uint32_t cap, bool pred, uint32_t key,
                                     float power) {
  const unsigned long long mask = __ballot(pred);
  if (mask == 0) return;
  const int lane = threadIdx.x % kWave;
  const int leader = __ffsll(static_cast<long long>(mask)) - 1;
  uint32_t base = 0;
  if (lane == leader && BRP_CHK(counter, sizeof(uint32_t))) base = atomicAdd(counter, static_cast<uint32_t>(__popcll(mask)));
  base = __shfl(base, leader, kWave);
  if (pred) {
    const uint32_t rank = __popcll(mask & ((1ull << lane) - 1ull));
    const uint32_t slot = base + rank;
    if (slot < cap) BRP_ST(&list[slot], make_uint2(key, __float_as_uint(power)));
  }
}

// MODE HS_F32: fp32 spectrum (exact path). HS_F16: fp16 spectrum (config 5),
// widened to float before the reference-order float sums.
//
// Each lane gathers the 16 harmonics of its index straight from global memory:
// within a wave the lanes of one harmonic read at most 4l+1 consecutive words
// (1-3 cache lines), and 10 workgroups per CU keep enough gathers in flight.
// (Measured alternatives -- LDS-staged runs, XCD-contiguous tiles, 4 or 16
// indices per lane, an MFMA selection-matrix sum -- are kept out of the
// product in tools/experiments/hs_variants.hip; profiles/hs_variants_r2.txt.)
//
// DENSE (the bounded-output path, launch_harmonic_sum_select): instead of
// emitting, every level value of [w2, fhi) is written to a.dense (0 where it
// does not exceed its threshold).
template <int MODE, bool DENSE = false>
__global__ void __launch_bounds__(kThreads) harmonic_sum_kernel(HSArgs a) {
#pragma clang fp contract(off)
  constexpr int TILE = kHsTile;
  static_assert(TILE % 16 == 0, "tiles start at i == 8 mod 16");
  constexpr int SPAN = TILE + kHalo;
  constexpr int SPAN_PAD = SPAN + SPAN / 16 + 1;
  constexpr bool kHalf = MODE != HS_F32;
  __shared__ __attribute__((aligned(16))) float lds[4 * SPAN_PAD];
  float (*sv)[SPAN_PAD] = reinterpret_cast<float (*)[SPAN_PAD]>(lds);
  const int b = blockIdx.y;
  const float* P32 = a.ps + static_cast<size_t>(b) * a.ps_stride;
  const _Float16* P16 = a.ps16 + static_cast<size_t>(b) * a.ps_stride;
  // signed: for windows below 16 the first tile starts before bin 0
  const int i0 = a.i_start + static_cast<int>(blockIdx.x) * TILE;
  const int w2 = static_cast<int>(a.w2), fhi = static_cast<int>(a.fhi), hhi = static_cast<int>(a.hhi);
  const float ninf = -__builtin_inff();
  // Gathers through a buffer descriptor: per harmonic l the thread computes
  // its bin offset once, (l (i0 + t) + 8) >> 4; iteration it (index + 256 it)
  // adds exactly 16 l it bins, an immediate of the load instruction. The
  // descriptor's range check turns the first tile's negative indices (windows
  // below 16) into zero reads.
  constexpr uint32_t kEsz = kHalf ? 2u : 4u;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      kHalf ? static_cast<void*>(const_cast<_Float16*>(P16)) : static_cast<void*>(const_cast<float*>(P32)), 0,
      static_cast<int>(a.ps_stride * kEsz), 0x00020000);
  // the descriptor's whole range lies in the spectrum allocation
  if (threadIdx.x == 0)
    (void)BRP_CHK(kHalf ? static_cast<const void*>(P16) : static_cast<const void*>(P32), a.ps_stride * kEsz);
  const int ib = i0 + static_cast<int>(threadIdx.x);
  uint32_t off[17];
#pragma unroll
  for (int l = 1; l <= 16; ++l) off[l] = kEsz * static_cast<uint32_t>((l * ib + 8) >> 4);
  auto ld = [&](int l, int it) -> float {
    const uint32_t o = off[l] + kEsz * 16u * static_cast<uint32_t>(l * it);
    if constexpr (kHalf) {
      const unsigned short bits = __builtin_amdgcn_raw_buffer_load_b16(rs, o, 0, 0);
      return static_cast<float>(__builtin_bit_cast(_Float16, bits));
    } else {
      return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, o, 0, 0));
    }
  };

  constexpr int kIt = (SPAN + kThreads - 1) / kThreads;
  float s1[kIt], s2[kIt], s3[kIt], s4[kIt], p0[kIt];
#pragma unroll
  for (int it = 0; it < kIt; ++it) {
    const int t = threadIdx.x + it * kThreads;
    const int i = i0 + t;
    s1[it] = s2[it] = s3[it] = s4[it] = ninf;
    p0[it] = 0.0f;
    if (t < SPAN && i >= w2 && i < hhi) {
      float sum = ld(16, it);
      p0[it] = sum;
      sum += ld(8, it);
      s1[it] = sum;
      sum += ld(12, it) + ld(4, it);
      s2[it] = sum;
      sum += ld(14, it) + ld(10, it) + ld(6, it) + ld(2, it);
      s3[it] = sum;
      sum += ld(15, it) + ld(13, it) + ld(11, it) + ld(9, it) + ld(7, it) + ld(5, it) + ld(3, it) + ld(1, it);
      s4[it] = sum;
    }
  }
#pragma unroll
  for (int it = 0; it < kIt; ++it) {
    const int t = threadIdx.x + it * kThreads;
    if (t < SPAN) {
      sv[0][sidx(t)] = s1[it];
      sv[1][sidx(t)] = s2[it];
      sv[2][sidx(t)] = s3[it];
      sv[3][sidx(t)] = s4[it];
    }
  }
  __syncthreads();

  uint32_t* count = &a.list[0].x;
  uint2* list = a.list + 1;
  const float thr0 = BRP_LD(&a.thr[static_cast<size_t>(b) * kHsThrStride + 0]);
  // level 0: the power spectrum itself (kept in registers from the S_1 sums)
#pragma unroll
  for (int it = 0; it < kIt; ++it) {
    const int t = threadIdx.x + it * kThreads;
    if (t - static_cast<int>(threadIdx.x) >= TILE) break;  // uniform: whole iterations past the tile
    const int i = i0 + t;
    const bool in = t < TILE && (i >= w2 && i < fhi);
    const float p = in ? p0[it] : 0.0f;
    if constexpr (DENSE) {
      if (in) BRP_ST(&a.dense[(static_cast<size_t>(b) * 5 + 0) * a.dense_stride + i], p > thr0 ? p : 0.0f);
    } else {
      emit(count, list, a.cap, in && p > thr0, hs_pack(a.key_base + b, 0, static_cast<uint32_t>(i), a.bin_bits), p);
    }
  }
  // levels 1..4: group of 2^h consecutive i starting at s == 2^(h-1) mod 2^h;
  // one thread per group, stride-2^h reads made (nearly) conflict free by the
  // t + t/16 padding of sv
#pragma unroll
  for (int h = 1; h <= 4; ++h) {
    const int g = 1 << h;
    const int off = g >> 1;
    const float thr = BRP_LD(&a.thr[static_cast<size_t>(b) * kHsThrStride + h]);
    const int first = static_cast<int>((off - (i0 % g) + g) % g);
    const int ngroups = (TILE - first + g - 1) / g;
    for (int q = threadIdx.x; q < ((ngroups + kThreads - 1) / kThreads) * kThreads; q += kThreads) {
      bool pred = false, inr = false;
      int j = 0;
      float m = ninf;
      if (q < ngroups) {
        const int t0 = first + q * g;
        j = (i0 + t0 + off) >> h;  // arithmetic shift: negative groups stay below w2
        if (j >= w2 && j < fhi) {
          inr = true;
#pragma unroll
          for (int u = 0; u < 16; ++u)
            if (u < g) m = fmaxf(m, sv[h - 1][sidx(t0 + u)]);
          pred = m > thr;
        }
      }
      if constexpr (DENSE) {
        if (inr) BRP_ST(&a.dense[(static_cast<size_t>(b) * 5 + h) * a.dense_stride + j], pred ? m : 0.0f);
      } else {
        emit(count, list, a.cap, pred, hs_pack(a.key_base + b, h, static_cast<uint32_t>(j), a.bin_bits), m);
      }
    }
  }
}

// ------------------------------------------------------------ pruned path
// The emission thresholds sit far above almost every harmonic sum (the
// chi^2 false-alarm levels of the reference, or the table floor once it is
// full), so the exact sums are only needed where some sum can reach one.
// Float addition is monotonic (a <= a', b <= b' => fl(a+b) <= fl(a'+b')), so
// summing, in the reference order, the maximum of every harmonic over the
// bins a 16-index block touches gives an upper bound of every level value the
// block owns; blocks whose bounds all stay at or below their thresholds emit
// nothing and are skipped. Harmonics 4..16 take their maxima from 8-bin cells
// (hs_cells_kernel; 4-bin cells as a switch), 1..3 from the spectrum: a wave's
// 64 blocks read ~1500 contiguous words instead of 16 x 1024 gathers. On the
// benchmark spectrum at the chi^2 thresholds about 1.2 % of the blocks pass
// (level 4; tools/experiments/hs_bound_sim.py, profiles/hs_bound_sim_r2.jsonl); those are then
// computed exactly like harmonic_sum_kernel does, so the candidate lists are
// the same (tests/test_gpu_kernels.py, bit for bit against the CPU model).
constexpr int kBlk = 16;      // indices per block: one level-4 group
constexpr int kBlkSpan = 20;  // + the 4-index reach of the level-1..3 groups whose first index lies in it
constexpr int kWaveSpan = kWave * kBlk + (kBlkSpan - kBlk);  // indices a wave's 64 blocks reach

// spectrum element type of a mode (HS_F16: fp16 spectrum, widened exactly)
template <int MODE>
using PsT = std::conditional_t<MODE == HS_F32, float, _Float16>;
template <int MODE>
__device__ __forceinline__ const PsT<MODE>* ps_row(const HSArgs& a, int b) {
  if constexpr (MODE == HS_F32) return a.ps + static_cast<size_t>(b) * a.ps_stride;
  else return a.ps16 + static_cast<size_t>(b) * a.ps_stride;
}

// maxima of the spectrum over cells of 2^CK bins (fp32 cells for either
// spectrum). REST (a.cells_ready, 8-bin cells): only the cells pass 3 did not
// write -- residues >= C/2 of the rows k3 < L3 (thread u -> row u / (C/16)),
// then every cell from M/8 on
template <int CK, int MODE, bool REST = false>
__global__ void __launch_bounds__(256) hs_cells_kernel(HSArgs a) {
  constexpr int W = 1 << CK;
  const int b = blockIdx.y;
  uint32_t m = blockIdx.x * 256u + threadIdx.x;
  if constexpr (REST) {
    const uint32_t per = a.row_c >> 4, nm = per * a.row_l;
    m = m < nm ? (m / per) * (a.row_c >> 3) + per + m % per : (a.row_c >> 3) * a.row_l + (m - nm);
  }
  if (m >= (a.ps_stride >> CK) + 8) return;
  const PsT<MODE>* P = ps_row<MODE>(a, b);
  const uint32_t k0 = W * m;
  float v[W];
  if (k0 + W <= a.hhi) {
    if constexpr (MODE == HS_F32) {
#pragma unroll
      for (int e = 0; e < W / 4; ++e) {
        const float4 x = BRP_LD(&reinterpret_cast<const float4*>(P + k0)[e]);
        v[4 * e] = x.x; v[4 * e + 1] = x.y; v[4 * e + 2] = x.z; v[4 * e + 3] = x.w;
      }
    } else {
#pragma unroll
      for (int e = 0; e < W / 4; ++e) {  // 4 halves per 8-byte load
        const uint2 x = BRP_LD(&reinterpret_cast<const uint2*>(P + k0)[e]);
        const uint32_t w[2] = {x.x, x.y};
#pragma unroll
        for (int q = 0; q < 4; ++q)
          v[4 * e + q] = static_cast<float>(
              __builtin_bit_cast(_Float16, static_cast<unsigned short>(w[q / 2] >> (16 * (q % 2)))));
      }
    }
  } else {
#pragma unroll
    for (int e = 0; e < W; ++e)  // never read by the exact sums
      v[e] = (k0 + e < a.hhi) ? static_cast<float>(BRP_LD(&P[k0 + e])) : 0.0f;
  }
#pragma unroll
  for (int w = W / 2; w >= 1; w /= 2)
#pragma unroll
    for (int e = 0; e < w; ++e) v[e] = fmaxf(v[e], v[e + w]);
  BRP_ST(&a.pyr[BRP_INJECT_AT(static_cast<size_t>(b) * a.pyr_stride + m, static_cast<size_t>(gridDim.y) * a.pyr_stride + 16,
                               kInjHsCells)],
         v[0]);
}

// 8-bin cells of an fp32 spectrum, CPT cells per thread (cells m0 + 256 j):
// all 2 CPT float4 loads are issued before the first maximum (one wave keeps
// 8 KB in flight instead of 2 KB; the one-cell kernel spent 81 % of its wave
// time waiting, profiles/hs_pmc_r6.txt). Cells reaching past hhi take the
// guarded per-bin path; their unconditional loads read bin 0 instead.
template <int CPT>
__global__ void __launch_bounds__(256) hs_cells8_kernel(HSArgs a) {
  const int b = blockIdx.y;
  const uint32_t n = (a.ps_stride >> 3) + 8;
  const uint32_t m0 = blockIdx.x * (256u * CPT) + threadIdx.x;
  const float* P = a.ps + static_cast<size_t>(b) * a.ps_stride;
  float4 x[CPT][2];
#pragma unroll
  for (int j = 0; j < CPT; ++j) {
    const uint32_t m = m0 + 256u * j, k0 = 8u * m;
    const uint32_t ks = (m < n && k0 + 8 <= a.hhi) ? k0 : 0u;
    x[j][0] = BRP_LD(reinterpret_cast<const float4*>(P + ks));
    x[j][1] = BRP_LD(reinterpret_cast<const float4*>(P + ks) + 1);
  }
#pragma unroll
  for (int j = 0; j < CPT; ++j) {
    const uint32_t m = m0 + 256u * j, k0 = 8u * m;
    if (m >= n) break;
    float v;
    if (k0 + 8 <= a.hhi) {
      v = fmaxf(fmaxf(fmaxf(x[j][0].x, x[j][1].x), fmaxf(x[j][0].y, x[j][1].y)),
                fmaxf(fmaxf(x[j][0].z, x[j][1].z), fmaxf(x[j][0].w, x[j][1].w)));
    } else {
      float t[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) t[e] = (k0 + e < a.hhi) ? BRP_LD(&P[k0 + e]) : 0.0f;
#pragma unroll
      for (int w = 4; w >= 1; w /= 2)
#pragma unroll
        for (int e = 0; e < w; ++e) t[e] = fmaxf(t[e], t[e + w]);
      v = t[0];
    }
    BRP_ST(&a.pyr[BRP_INJECT_AT(static_cast<size_t>(b) * a.pyr_stride + m,
                                static_cast<size_t>(gridDim.y) * a.pyr_stride + 16, kInjHsCells)],
           v);
  }
}

// harmonics in the reference summation order, their source (0: spectrum,
// CK: 2^CK-bin cells) and their slice of a wave's staging buffer
constexpr int kHarm[16] = {16, 8, 12, 4, 14, 10, 6, 2, 15, 13, 11, 9, 7, 5, 3, 1};
template <int CK>
struct HsStage {
  static constexpr int lvl(int l) { return l >= 4 ? CK : 0; }
  // cells of harmonic l the wave's blocks reach, counted from the wave's first
  // cell rounded down to even (so that cell pairs are 8-byte aligned in LDS)
  static constexpr int wave_cells(int l) { return (((l * (kWaveSpan - 1) + 15) / 16) >> lvl(l)) + 3; }
  static constexpr int slice_len(int l) { return (wave_cells(l) + 1) & ~1; }
  static constexpr int slice(int q) {
    int o = 0;
    for (int r = 0; r < q; ++r) o += slice_len(kHarm[r]);
    return o;
  }
  static constexpr int kCells = slice(16) + 8;  // pair reads past a slice end stay inside the buffer
  static constexpr int chunks(int q) { return (slice_len(kHarm[q]) + kWave - 1) / kWave; }
  static constexpr int chunk0(int q) {
    int o = 0;
    for (int r = 0; r < q; ++r) o += chunks(r);
    return o;
  }
  static constexpr int kLoads = chunk0(16);
};

__device__ __forceinline__ uint32_t hs_cell(int l, int k, int32_t i) {
  return (static_cast<uint32_t>(l * (i < 0 ? 0 : i) + 8) >> 4) >> k;
}

// the cells harmonic kHarm[Q] of the wave's blocks reach, contiguous: every
// lane loads its words of all 16 slices first (unconditional, clamped
// addresses: a guarded load per word made the compiler wait for each one
// before its LDS write), then writes them to the wave's staging buffer
template <int CK, int Q, typename T>
__device__ __forceinline__ void hs_load(float* v, const T* P, const float* C8, uint32_t n8, uint32_t nps,
                                        int32_t I0, int lane) {
  using S = HsStage<CK>;
  constexpr int L = kHarm[Q], K = S::lvl(L);
  const uint32_t lim = K ? n8 : nps;
  const uint32_t c0 = hs_cell(L, K, I0) & ~1u;
#pragma unroll
  for (int q = 0; q < S::chunks(Q); ++q) {
    const uint32_t c = c0 + static_cast<uint32_t>(lane + kWave * q);
    const float x = K ? BRP_LD(&C8[min(c, lim - 1)]) : static_cast<float>(BRP_LD(&P[min(c, lim - 1)]));
    v[S::chunk0(Q) + q] = c < lim ? x : 0.0f;
  }
}

template <int CK, int Q>
__device__ __forceinline__ void hs_store(float* buf, const float* v, int lane) {
  using S = HsStage<CK>;
  constexpr int N = S::slice_len(kHarm[Q]);
#pragma unroll
  for (int q = 0; q < S::chunks(Q); ++q) {
    const int e = lane + kWave * q;
    if (e < N) buf[S::slice(Q) + e] = v[S::chunk0(Q) + q];
  }
}

// max of harmonic kHarm[Q] over the N indices [i, i + N) from the staged cells
template <int CK, int Q, int N>
__device__ __forceinline__ float hs_span_max(const float* buf, int32_t I0, int32_t i) {
  using S = HsStage<CK>;
  constexpr int L = kHarm[Q], K = S::lvl(L);
  constexpr int kCells = (((L * (N - 1) + 15) / 16) >> K) + 2;
  const float* s = buf + S::slice(Q) - (hs_cell(L, K, I0) & ~1u);
  const uint32_t lo = hs_cell(L, K, i), hi = hs_cell(L, K, i + N - 1);
  float m = s[lo];
#pragma unroll
  for (int d = 1; d < kCells; ++d) m = fmaxf(m, s[min(lo + d, hi)]);
  return m;
}

template <int CK, typename T, int... Q>
__device__ __forceinline__ void hs_stage_all(std::integer_sequence<int, Q...>, float* buf, const T* P,
                                             const float* C8, uint32_t n8, uint32_t nps, int32_t I0, int lane) {
  float v[HsStage<CK>::kLoads];
  (hs_load<CK, Q>(v, P, C8, n8, nps, I0, lane), ...);
  (hs_store<CK, Q>(buf, v, lane), ...);
}

// level bounds of block [ib, ib + 16) in the reference summation order (see
// harmonic_sum_kernel). Level 4 owns one group, exactly the block's 16
// indices; the groups of levels 1..3 whose first index lies in the block reach
// 4 indices further, so their harmonics (the first 8) also take the max over
// [ib + 16, ib + 20). (Measured on the benchmark spectrum with the chi^2
// thresholds, tools/experiments/hs_bound_sim.py: level 4 decides almost every
// flag; its own 16-index span halves the flagged blocks against one 20-index
// span for all levels, 4-bin cells halve them again.)
template <int CK, int... Q>
__device__ __forceinline__ void hs_tail_max(std::integer_sequence<int, Q...>, const float* buf, int32_t I0, int32_t i,
                                            float* m) {
  ((m[Q] = fmaxf(m[Q], hs_span_max<CK, Q, kBlkSpan - kBlk>(buf, I0, i))), ...);
}

// Maxima of harmonic kHarm[Q] over the block's 16 indices (m16) and, for the
// first 8 harmonics, over its 20-index reach (m20), read as aligned cell pairs
// (ds_read_b64). A 32-lane group of b64 reads is serviced by 64 banks, and the
// pairs lanes request advance by L/16 <= 1 per lane (8-bin cells), so the reads
// are conflict free; b32 reads of the same cells advance by L/8 > 1 words per
// lane for L > 8 and collided 2-way (profiles/pmc_bytes_pruned_hs_r2.txt: 62 %
// of the kernel's LDS cycles were bank conflicts). Cells outside [lo, hi] of
// the loaded pairs are masked, so the maxima (and the bounds) are exactly
// those of hs_span_max. Harmonic 3 reads spectrum words at a stride of 3 per
// lane: b32 reads are already conflict free there (pairs would not be).
template <int CK, int Q>
__device__ __forceinline__ void hs_pair_max(const float* buf, int32_t I0, int32_t ib, float& m16, float& m20) {
  using S = HsStage<CK>;
  constexpr int L = kHarm[Q], K = S::lvl(L);
  constexpr bool kTail = Q < 8;
  if constexpr (L == 3) {
    m16 = m20 = hs_span_max<CK, Q, kBlk>(buf, I0, ib);
  } else {
    constexpr int N = kTail ? kBlkSpan : kBlk;
    constexpr int kSpan = (((L * (N - 1) + 15) / 16) >> K) + 2;  // hi - lo < kSpan
    constexpr int NP = kSpan / 2 + 1;                              // pairs covering [lo & ~1, lo + kSpan)
    const float ninf = -__builtin_inff();
    const uint32_t cb = hs_cell(L, K, I0) & ~1u;
    const uint32_t lo = hs_cell(L, K, ib), h16 = hs_cell(L, K, ib + kBlk - 1);
    const uint32_t h20 = kTail ? hs_cell(L, K, ib + kBlkSpan - 1) : h16;
    // volatile: keeps each pair read a ds_read_b64 (the load-store optimiser
    // would merge neighbours into ds_read2_b64, serviced as 32 banks / 4 x 16
    // lanes at twice the cycles)
    using f2 = float __attribute__((ext_vector_type(2)));
    using lds_f2 = const volatile f2 __attribute__((address_space(3)))*;
    const lds_f2 s = (lds_f2)(buf + S::slice(Q)) + ((lo - cb) >> 1);
    const uint32_t c0 = lo & ~1u;
    // cells c0 + e with e <= kIn lie in [lo, h16] for every block: since
    // (x + y) >> 4 >= (x >> 4) + (y >> 4), h16 - lo >= (15 L / 16) >> K
    constexpr int kIn = ((15 * L) / 16) >> K;
    float a = ninf, t = ninf;
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      const f2 v = s[j];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int i = 2 * j + e;
        float x = e ? v.y : v.x;
        if (i == 0) x = (lo & 1u) ? ninf : x;
        if (i <= kIn) {
          a = fmaxf(a, x);
        } else {
          const uint32_t c = c0 + static_cast<uint32_t>(i);
          a = fmaxf(a, c <= h16 ? x : ninf);
          if constexpr (kTail) t = fmaxf(t, c <= h20 ? x : ninf);
        }
      }
    }
    t = fmaxf(a, t);
    m16 = a;
    m20 = kTail ? t : a;
  }
}

// The same maxima read straight from global memory, without LDS staging:
// for every harmonic the bins (l < 4) or 8-bin cells (l >= 4) a block reaches
// lie in the 4 consecutive entries from lo (hi - lo <= 3, checked below), so
// one 16-byte load per harmonic and lane covers them (the loads of a wave
// overlap: the cache serves them). No LDS is held while the loads are in
// flight, so the pass kernels running beside this one keep their occupancy.
template <int CK, int Q>
struct HsDirect {
  static constexpr int L = kHarm[Q], K = HsStage<CK>::lvl(L);
  static constexpr bool kTail = Q < 8;
  // largest hi - lo over all blocks for a span of N indices
  static constexpr int kD16 = ((((L * (kBlk - 1) + 15) / 16) + (1 << K) - 1) >> K);
  static constexpr int kD20 = ((((L * (kBlkSpan - 1) + 15) / 16) + (1 << K) - 1) >> K);
  static_assert((kTail ? kD20 : kD16) <= 3, "one load of at most 4 entries per harmonic");
  static constexpr int kIn = ((15 * L) / 16) >> K;  // entries e <= kIn lie in [lo, h16] for every block
  static constexpr int kN = (kTail ? kD20 : kD16) + 1;  // entries a block can reach (1..4)
};

// N consecutive floats from a dword-aligned address as one load
template <int N>
using fvu = float __attribute__((ext_vector_type(N), aligned(4)));
using f4u = fvu<4>;

// the entries from lo of harmonic kHarm[Q] a block can reach, as one load of
// exactly that many dwords (45 instead of 64 VGPRs for the 16 harmonics)
template <int CK, int Q, int MODE>
__device__ __forceinline__ f4u hs_direct_load(const PsT<MODE>* P, const float* C8, int32_t ib) {
  using H = HsDirect<CK, Q>;
  const uint32_t lo = hs_cell(H::L, H::K, ib);
  f4u v = {0.0f, 0.0f, 0.0f, 0.0f};
  if constexpr (H::K > 0 || MODE == HS_F32) {
    const float* src = (H::K > 0 ? C8 : reinterpret_cast<const float*>(P)) + lo;
    if constexpr (H::kN == 1) {
      v.x = BRP_LD(src);
    } else {
      const fvu<H::kN> w = BRP_LD(reinterpret_cast<const fvu<H::kN>*>(src));
#pragma unroll
      for (int e = 0; e < H::kN; ++e) v[e] = w[e];
    }
  } else {
#pragma unroll
    for (int e = 0; e < H::kN; ++e) v[e] = static_cast<float>(BRP_LD(&P[lo + e]));
  }
  return v;
}

// maxima over the block's 16 indices (m16) and, for the first 8 harmonics,
// its 20-index reach (m20) from the loaded entries; entries past h16 / h20
// are masked
template <int CK, int Q>
__device__ __forceinline__ void hs_direct_max(f4u v, int32_t ib, float& m16, float& m20) {
  using H = HsDirect<CK, Q>;
  const uint32_t lo = hs_cell(H::L, H::K, ib), h16 = hs_cell(H::L, H::K, ib + kBlk - 1);
  const uint32_t h20 = H::kTail ? hs_cell(H::L, H::K, ib + kBlkSpan - 1) : h16;
  const float x[4] = {v.x, v.y, v.z, v.w};
  const float ninf = -__builtin_inff();
  const uint32_t d16 = h16 - lo, d20 = h20 - lo;
  float a = x[0], t = ninf;
#pragma unroll
  for (int e = 1; e <= (H::kTail ? H::kD20 : H::kD16); ++e) {
    if (e <= H::kIn) {
      a = fmaxf(a, x[e]);
    } else {
      if (e <= H::kD16) a = fmaxf(a, static_cast<uint32_t>(e) <= d16 ? x[e] : ninf);
      if constexpr (H::kTail) t = fmaxf(t, static_cast<uint32_t>(e) <= d20 ? x[e] : ninf);
    }
  }
  m16 = a;
  m20 = H::kTail ? fmaxf(a, t) : a;
}

// Bounds from direct reads: all 16 loads issued before the first use (with
// the ordering pins the staged path needs, the compiler waited for each pair
// of loads in turn: ~8 memory latencies per wave); sums in the reference
// order as in hs_bounds.
template <int CK, int MODE, int... Q>
__device__ __forceinline__ void hs_bounds_direct(std::integer_sequence<int, Q...>, const PsT<MODE>* P,
                                                 const float* C8, int32_t ib, float* u) {
  const f4u v[16] = {hs_direct_load<CK, Q, MODE>(P, C8, ib)...};
  // every load in flight before the first is consumed (the scheduler otherwise
  // splits them into two rounds around the first maxima)
  auto issued = [](f4u x) { asm volatile("" ::"v"(x)); };
  (issued(v[Q]), ...);
  float m16[16], m20[16];
  (hs_direct_max<CK, Q>(v[Q], ib, m16[Q], m20[Q]), ...);
  u[0] = m20[0];
  u[1] = u[0] + m20[1];
  u[2] = u[1] + (m20[2] + m20[3]);
  u[3] = u[2] + (((m20[4] + m20[5]) + m20[6]) + m20[7]);
  float w0 = m16[0];
  w0 += m16[1];
  w0 += m16[2] + m16[3];
  w0 += ((m16[4] + m16[5]) + m16[6]) + m16[7];
  float w = m16[8] + m16[9];
  w = (w + m16[10]) + m16[11];
  w = (w + m16[12]) + m16[13];
  w = (w + m16[14]) + m16[15];
  u[4] = w0 + w;
}

template <int CK, bool DIRECT, int MODE, int... Q>
__device__ __forceinline__ void hs_bounds(std::integer_sequence<int, Q...>, const float* buf, const PsT<MODE>* P,
                                          const float* C8, int32_t I0, int32_t ib, float* u) {
  if constexpr (CK == 3) {
    // running sums in the reference order, harmonic by harmonic; each group's
    // partial sums are pinned (empty volatile asm) before the next group's
    // volatile pair reads, so the reads of one group die before the next are
    // issued (all 33 hoisted ahead of their uses held 120 VGPRs: 4 instead of
    // 5 waves per SIMD)
    float m16, m20, x16, x20;
    auto hm = [&](auto qc, float& a16, float& a20) {
      hs_pair_max<CK, decltype(qc)::value>(buf, I0, ib, a16, a20);
    };
    using std::integral_constant;
    auto pin = [](float& p, float& q) { asm volatile("" : "+v"(p), "+v"(q)); };
    hm(integral_constant<int, 0>{}, m16, m20);
    u[0] = m20;
    float v = m16;
    hm(integral_constant<int, 1>{}, m16, m20);
    u[1] = u[0] + m20;
    v += m16;
    pin(u[1], v);
    hm(integral_constant<int, 2>{}, m16, m20);
    hm(integral_constant<int, 3>{}, x16, x20);
    u[2] = u[1] + (m20 + x20);
    v += m16 + x16;
    pin(u[2], v);
    hm(integral_constant<int, 4>{}, m16, m20);
    hm(integral_constant<int, 5>{}, x16, x20);
    float s20 = m20 + x20, s16 = m16 + x16;
    pin(s20, s16);
    hm(integral_constant<int, 6>{}, m16, m20);
    hm(integral_constant<int, 7>{}, x16, x20);
    u[3] = u[2] + ((s20 + m20) + x20);
    v += (s16 + m16) + x16;
    pin(u[3], v);
    hm(integral_constant<int, 8>{}, m16, m20);
    hm(integral_constant<int, 9>{}, x16, x20);
    float w = m16 + x16;
    pin(w, v);
    hm(integral_constant<int, 10>{}, m16, m20);
    hm(integral_constant<int, 11>{}, x16, x20);
    w = (w + m16) + x16;
    pin(w, v);
    hm(integral_constant<int, 12>{}, m16, m20);
    hm(integral_constant<int, 13>{}, x16, x20);
    w = (w + m16) + x16;
    pin(w, v);
    hm(integral_constant<int, 14>{}, m16, m20);
    hm(integral_constant<int, 15>{}, x16, x20);
    w = (w + m16) + x16;
    u[4] = v + w;
    (void)m20;
    (void)x20;
  } else {  // 4-bin cells (switch): pair strides of 2 would collide; b32 reads
    (void)P;
    (void)C8;
    const float m16[16] = {hs_span_max<CK, Q, kBlk>(buf, I0, ib)...};
    float m20[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) m20[q] = m16[q];
    hs_tail_max<CK>(std::make_integer_sequence<int, 8>{}, buf, I0, ib + kBlk, m20);
    u[0] = m20[0];
    u[1] = u[0] + m20[1];
    u[2] = u[1] + (m20[2] + m20[3]);
    u[3] = u[2] + (((m20[4] + m20[5]) + m20[6]) + m20[7]);
    float v = m16[0];
    v += m16[1];
    v += m16[2] + m16[3];
    v += ((m16[4] + m16[5]) + m16[6]) + m16[7];
    u[4] = v + (((((((m16[8] + m16[9]) + m16[10]) + m16[11]) + m16[12]) + m16[13]) + m16[14]) + m16[15]);
  }
}

// One thread per 16-index block computes the bounds; the wave then computes
// its flagged blocks exactly, three at a time (lanes 20 s .. 20 s + 19 hold
// indices ib .. ib + 19 of block s), with the sums, level maxima and emission
// of harmonic_sum_kernel for the groups whose first index lies in the block.
// (No global block list: an atomic per wave on one counter serialised a first
// version at 39 us.)
template <int CK, int MODE, bool DIRECT>
__global__ void __launch_bounds__(256) hs_pruned_kernel(HSArgs a, uint32_t nblk) {
#pragma clang fp contract(off)
  static_assert(!DIRECT || CK == 3, "direct bound reads: 8-bin cells");
  constexpr int kSubs = kWave / kBlkSpan;  // 3
  __shared__ __attribute__((aligned(16))) float stage[DIRECT ? 1 : 4][DIRECT ? 4 : HsStage<CK>::kCells];
  __shared__ float sv[4][kSubs][4][kBlkSpan];
  const int b = blockIdx.y;
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const uint32_t bx = a.xcd ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
  const uint32_t wave_blk0 = bx * 256u + static_cast<uint32_t>(wave * kWave);
  if (wave_blk0 >= nblk) return;  // whole wave
#ifdef BRP_ABLATE_HS
  return;  // speed-of-light ablation (experiment builds only: no candidates)
#endif
  const uint32_t blk = wave_blk0 + lane;
  const PsT<MODE>* P = ps_row<MODE>(a, b);
  const float* thr = a.thr + static_cast<size_t>(b) * kHsThrStride;
  const int w2 = static_cast<int>(a.w2), fhi = static_cast<int>(a.fhi), hhi = static_cast<int>(a.hhi);
  const int32_t I0 = a.i_start + static_cast<int32_t>(kBlk * wave_blk0);
  float* buf = stage[DIRECT ? 0 : wave];
  const float* C8 = a.pyr + BRP_INJECT_AT(static_cast<size_t>(b) * a.pyr_stride,
                                          static_cast<size_t>(gridDim.y) * a.pyr_stride + 16, kInjHsPruned);
  if constexpr (!DIRECT) hs_stage_all<CK>(std::make_integer_sequence<int, 16>{}, buf, P, C8, a.pyr_stride, a.ps_stride, I0, lane);
  // LDS operations of one wave complete in order; keep the compiler from moving them
  auto wave_sync = [] {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_wave_barrier();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
  };
  wave_sync();
#ifdef BRP_ABLATE_HS_STAGE
  if (buf[lane] == -1.0f) a.list[1].x = 0;  // keep the staging live; never true for powers
  return;  // ablation: staging only
#endif
  bool flag = false;
  // the five thresholds up front (uniform: scalar loads), not one guarded load
  // per level after the bounds
  float th[5];
#pragma unroll
  for (int h = 0; h <= 4; ++h) th[h] = BRP_LD(&thr[h]);
  if (blk < nblk) {
    const int32_t ib = I0 + kBlk * lane;
    float u[5];
    if constexpr (DIRECT) hs_bounds_direct<CK, MODE>(std::make_integer_sequence<int, 16>{}, P, C8, ib, u);
    else hs_bounds<CK, DIRECT, MODE>(std::make_integer_sequence<int, 16>{}, buf, P, C8, I0, ib, u);
#pragma unroll
    for (int h = 0; h <= 4; ++h) {
      const int off = h ? 1 << (h - 1) : 0;
      const int j_lo = (ib + off) >> h, j_hi = (ib + kBlk - 1 + off) >> h;  // groups whose first index is in the block
      flag |= (j_hi >= w2 && j_lo < fhi) && !(u[h] <= th[h]);              // NaN bounds are kept
    }
  }
  unsigned long long mask = __ballot(flag);
#ifdef BRP_ABLATE_HS_EXACT
  if (mask != 0 && lane == 0 && thr[0] < 0.0f) a.list[1].x = 0;  // keep the bounds live
  return;  // ablation: staging + bounds, no exact sums
#endif
  if (mask == 0) return;

  const int sub = lane / kBlkSpan, li = lane % kBlkSpan;
  const float ninf = -__builtin_inff();
  uint32_t* count = &a.list[0].x;
  uint2* list = a.list + 1;
  while (mask != 0) {  // wave-uniform
    // the next three flagged blocks of the wave go to subs 0, 1, 2
    int bit = -1;
#pragma unroll
    for (int s = 0; s < kSubs; ++s) {
      const int f = mask ? __ffsll(static_cast<long long>(mask)) - 1 : -1;
      if (f >= 0) mask &= mask - 1;
      if (s == sub) bit = f;
    }
    const bool act = sub < kSubs && bit >= 0;
    const int32_t ib = I0 + kBlk * (act ? bit : 0);
    const int i = ib + li;
    float s1 = ninf, s2 = ninf, s3 = ninf, s4 = ninf, p0 = 0.0f;
    if (act && i >= w2 && i < hhi) {
      auto ld = [&](int l) { return static_cast<float>(BRP_LD(&P[(l * i + 8) >> 4])); };
      float sum = ld(16);
      p0 = sum;
      sum += ld(8);
      s1 = sum;
      sum += ld(12) + ld(4);
      s2 = sum;
      sum += ld(14) + ld(10) + ld(6) + ld(2);
      s3 = sum;
      sum += ld(15) + ld(13) + ld(11) + ld(9) + ld(7) + ld(5) + ld(3) + ld(1);
      s4 = sum;
    }
    if (sub < kSubs) {
      sv[wave][sub][0][li] = s1;
      sv[wave][sub][1][li] = s2;
      sv[wave][sub][2][li] = s3;
      sv[wave][sub][3][li] = s4;
    }
    wave_sync();
    // level 0: the spectrum itself, indices of the block
    const bool in0 = act && li < kBlk && i >= w2 && i < fhi;
    emit(count, list, a.cap, in0 && p0 > thr[0], hs_pack(a.key_base + b, 0, static_cast<uint32_t>(i), a.bin_bits), p0);
    // levels 1..4: lane li < 15 owns one group (8 of level 1, 4 of level 2, 2 of level 3, 1 of level 4)
    int h = 4, t0 = 0;
    if (li < 8) { h = 1; t0 = 2 * li + 1; }
    else if (li < 12) { h = 2; t0 = 4 * (li - 8) + 2; }
    else if (li < 14) { h = 3; t0 = 8 * (li - 12) + 4; }
    const int g = 1 << h;
    float m = ninf;
    bool pred = false;
    int j = 0;
    if (act && li < 15) {
      for (int q = 0; q < g; ++q) m = fmaxf(m, sv[wave][sub][h - 1][t0 + q]);
      j = (ib + t0 + (g >> 1)) >> h;
      pred = j >= w2 && j < fhi && m > thr[h];
    }
    emit(count, list, a.cap, pred,
         hs_pack(a.key_base + b, static_cast<uint32_t>(h), static_cast<uint32_t>(j), a.bin_bits), m);
    wave_sync();
  }
}


// ------------------------------------------------------------ bounded output
// Radix select of the K-th largest level value per (template, level) over
// the dense values of [w2, fhi): three rounds of 11 / 11 / 10 bits of the
// float bit pattern (positive floats order like their bits), each a histogram
// of the values matching the prefix found so far, then one wave picking the
// next digit. State per (template, level): prefix, K remaining, "fewer than K
// values above threshold" flag, number of such values.
constexpr int kSelShift[3] = {21, 10, 0};
constexpr int kSelBits[3] = {11, 11, 10};
constexpr uint32_t kSelChunk = 256 * 16;  // values per histogram workgroup

template <int ROUND>
__global__ void __launch_bounds__(256) hs_sel_hist_kernel(HSArgs a, HsSelectArgs s) {
  constexpr int kShift = kSelShift[ROUND], kBits = kSelBits[ROUND];
  __shared__ uint32_t hist[kHsSelBins];
  const uint32_t h = blockIdx.y, b = blockIdx.z;
  const size_t row = static_cast<size_t>(b) * 5 + h;
  const uint32_t* st = s.state + row * 4;
  if (threadIdx.x == 0) (void)BRP_CHK(st, 4 * sizeof(uint32_t));
  if (ROUND > 0 && st[2] != 0) return;  // uniform: fewer than K values, nothing to refine
  for (uint32_t e = threadIdx.x; e < (1u << kBits); e += 256) hist[e] = 0;
  __syncthreads();
  const uint32_t prefix = st[0];
  const uint32_t* v = reinterpret_cast<const uint32_t*>(s.dense) + row * s.dense_stride;
  const uint32_t lo = a.w2 + blockIdx.x * kSelChunk, hi = min(lo + kSelChunk, a.fhi);
  for (uint32_t j = lo + threadIdx.x; j < hi; j += 256) {
    const uint32_t u = BRP_LD(&v[j]);
    if (u == 0 || (u >> 31) != 0) continue;  // not above threshold
    if (ROUND > 0 && (u >> (kShift + kBits)) != (prefix >> (kShift + kBits))) continue;
    atomicAdd(&hist[(u >> kShift) & ((1u << kBits) - 1u)], 1u);
  }
  __syncthreads();
  uint32_t* g = s.hist + row * kHsSelBins;
  for (uint32_t e = threadIdx.x; e < (1u << kBits); e += 256)
    if (hist[e] != 0 && BRP_CHK(&g[e], sizeof(uint32_t))) atomicAdd(&g[e], hist[e]);
}

// one wave per (template, level): lane l owns bins [32 l, 32 l + 32)
template <int ROUND>
__global__ void __launch_bounds__(64) hs_sel_pick_kernel(HSArgs a, HsSelectArgs s) {
  constexpr int kShift = kSelShift[ROUND], kBits = kSelBits[ROUND];
  constexpr int kPer = (1 << kBits) / kWave;
  const uint32_t h = blockIdx.x, b = blockIdx.y;
  const size_t row = static_cast<size_t>(b) * 5 + h;
  uint32_t* st = s.state + row * 4;
  if (threadIdx.x == 0) (void)BRP_CHK(st, 4 * sizeof(uint32_t));
  uint32_t* g = s.hist + row * kHsSelBins;
  const int lane = threadIdx.x;
  if (ROUND > 0 && st[2] != 0) return;
  uint32_t mine[kPer];
  uint32_t sum = 0;
#pragma unroll
  for (int e = 0; e < kPer; ++e) {
    mine[e] = BRP_LD(&g[lane * kPer + e]);
    BRP_ST(&g[lane * kPer + e], 0u);  // cleared for the next round
    sum += mine[e];
  }
  // suffix sums over the lanes: values in the bins of lanes >= lane
  uint32_t suf = sum;
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) {
    const uint32_t o = __shfl_down(suf, off, kWave);
    if (lane + off < kWave) suf += o;
  }
  const uint32_t krem = st[1];
  const uint32_t total = __shfl(suf, 0, kWave);
  if (ROUND == 0) {
    if (lane == 0) {
      st[3] = total;
      if (BRP_CHK(&a.list[0].y, sizeof(uint32_t))) atomicAdd(&a.list[0].y, total);
    }
    if (total < krem) {  // fewer than K values above threshold: all of them are kept
      if (lane == 0) st[2] = 1;
      return;
    }
  }
  // the highest lane whose suffix still reaches krem holds the K-th value's digit
  const unsigned long long reach = __ballot(suf >= krem);
  const int L = 63 - __clzll(static_cast<long long>(reach));
  if (lane == L) {
    uint32_t above = suf - sum;  // values in higher lanes' bins
    int digit = 0;
    for (int e = kPer - 1; e >= 0; --e) {
      if (above + mine[e] >= krem) {
        digit = lane * kPer + e;
        break;
      }
      above += mine[e];
    }
    st[0] |= static_cast<uint32_t>(digit) << kShift;
    st[1] = krem - above;
  }
}

__global__ void hs_sel_init_kernel(uint32_t* state, uint32_t rows, uint32_t k) {
  const uint32_t r = blockIdx.x * 256u + threadIdx.x;
  if (r < rows) BRP_ST(&reinterpret_cast<uint4*>(state)[r], make_uint4(0u, k, 0u, 0u));
}

// emit every value >= the K-th largest (all of them when there are fewer than K)
__global__ void __launch_bounds__(256) hs_sel_emit_kernel(HSArgs a, HsSelectArgs s) {
  const uint32_t h = blockIdx.y, b = blockIdx.z;
  const size_t row = static_cast<size_t>(b) * 5 + h;
  const uint32_t* st = s.state + row * 4;
  if (threadIdx.x == 0) (void)BRP_CHK(st, 4 * sizeof(uint32_t));
  const uint32_t kth = st[2] != 0 ? 1u : st[0];
  const uint32_t* v = reinterpret_cast<const uint32_t*>(s.dense) + row * s.dense_stride;
  const uint32_t lo = a.w2 + blockIdx.x * kSelChunk, hi = min(lo + kSelChunk, a.fhi);
  uint32_t* count = &a.list[0].x;
  uint2* list = a.list + 1;
  // whole-wave iterations (emit aggregates with a ballot)
  for (uint32_t j0 = lo; j0 < hi; j0 += 256) {
    const uint32_t j = j0 + threadIdx.x;
    const uint32_t u = j < hi ? BRP_LD(&v[j]) : 0u;
    const bool keep = u != 0 && (u >> 31) == 0 && u >= kth;
    emit(count, list, a.cap, keep, hs_pack(a.key_base + b, h, j, a.bin_bits), __uint_as_float(u));
  }
}

}  // namespace

hipError_t preload_harmonic_sum() {
  hipFuncAttributes at;
  return hipFuncGetAttributes(&at, reinterpret_cast<const void*>(&hs_sel_init_kernel));
}

uint32_t hs_num_blocks(int32_t i_start, uint32_t hhi) {
  const int64_t span = static_cast<int64_t>(hhi) - i_start;
  if (span <= 0) return 0;
  return static_cast<uint32_t>((span + kBlk - 1) / kBlk);
}

uint32_t hs_num_tiles(int32_t i_start, uint32_t hhi) {
  const int64_t span = static_cast<int64_t>(hhi) - i_start;
  if (span <= 0) return 0;
  return static_cast<uint32_t>((span + kHsTile - 1) / kHsTile);
}

hipError_t launch_harmonic_sum(const HSArgs& a, int batch, hipStream_t s) {
  if (a.prune) {
    const uint32_t nblk = hs_num_blocks(a.i_start, a.hhi);
    if (nblk == 0) return hipSuccess;
    const dim3 gc((hs_pyr_stride(a.ps_stride) + 255) / 256, batch), gp((nblk + 255) / 256, batch);
    // cells pass 3 left (cells_ready): the mirror half of rows k3 < L3, then the cells from M/8 on
    const uint32_t n8 = (a.ps_stride >> 3) + 8, m8 = (a.row_c >> 3) * a.row_l;
    const uint32_t n_rest = (a.row_c >> 4) * a.row_l + (n8 > m8 ? n8 - m8 : 0u);
    const dim3 gr((n_rest + 255) / 256, batch), g4((n8 + 1023) / 1024, batch);
#define BRP_HS_PRUNED(CK, MODE, DIRECT)                                                    \
  do {                                                                                    \
    if (CK == 3 && a.cells_ready) BRP_LAUNCH((hs_cells_kernel<CK, MODE, true>), gr, dim3(256), 0, s, a); \
    else if (CK == 3 && MODE == HS_F32 && a.cells_cpt == 4) BRP_LAUNCH(hs_cells8_kernel<4>, g4, dim3(256), 0, s, a); \
    else BRP_LAUNCH((hs_cells_kernel<CK, MODE>), gc, dim3(256), 0, s, a);                \
    BRP_LAUNCH((hs_pruned_kernel<CK, MODE, DIRECT>), gp, dim3(256), 0, s, a, nblk);       \
  } while (0)
    if (a.mode == HS_F16) {
      if (a.cell_shift == 2) BRP_HS_PRUNED(2, HS_F16, false);
      else if (a.direct) BRP_HS_PRUNED(3, HS_F16, true);
      else BRP_HS_PRUNED(3, HS_F16, false);
    } else {
      if (a.cell_shift == 2) BRP_HS_PRUNED(2, HS_F32, false);
      else if (a.direct) BRP_HS_PRUNED(3, HS_F32, true);
      else BRP_HS_PRUNED(3, HS_F32, false);
    }
#undef BRP_HS_PRUNED
    return launch_status();
  }
  const uint32_t tiles = hs_num_tiles(a.i_start, a.hhi);
  if (tiles == 0) return hipSuccess;
  const dim3 grid(tiles, batch);
  switch (a.mode) {
    case HS_F16: BRP_LAUNCH(harmonic_sum_kernel<HS_F16>, grid, dim3(kThreads), 0, s, a); break;
    default: BRP_LAUNCH(harmonic_sum_kernel<HS_F32>, grid, dim3(kThreads), 0, s, a); break;
  }
  return launch_status();
}


hipError_t launch_harmonic_sum_select(const HSArgs& a0, const HsSelectArgs& s, int batch, hipStream_t st) {
  HSArgs a = a0;
  a.dense = s.dense;
  a.dense_stride = s.dense_stride;
  const uint32_t tiles = hs_num_tiles(a.i_start, a.hhi);
  if (a.fhi <= a.w2 || tiles == 0 || s.dense_stride < a.fhi) return hipSuccess;
  hipError_t e;
  const size_t rows = static_cast<size_t>(batch) * 5;
  if ((e = hipMemsetAsync(s.dense, 0, rows * s.dense_stride * sizeof(float), st)) != hipSuccess) return e;
  if ((e = hipMemsetAsync(s.hist, 0, rows * kHsSelBins * sizeof(uint32_t), st)) != hipSuccess) return e;
  const dim3 grid(tiles, batch);
  if (a.mode == HS_F16) BRP_LAUNCH((harmonic_sum_kernel<HS_F16, true>), grid, dim3(kThreads), 0, st, a);
  else BRP_LAUNCH((harmonic_sum_kernel<HS_F32, true>), grid, dim3(kThreads), 0, st, a);
  const dim3 gh((a.fhi - a.w2 + kSelChunk - 1) / kSelChunk, 5, batch), gp(5, batch);
  BRP_LAUNCH(hs_sel_init_kernel, dim3((rows + 255) / 256), dim3(256), 0, st, s.state,
                     static_cast<uint32_t>(rows), s.k);
  BRP_LAUNCH(hs_sel_hist_kernel<0>, gh, dim3(256), 0, st, a, s);
  BRP_LAUNCH(hs_sel_pick_kernel<0>, gp, dim3(64), 0, st, a, s);
  BRP_LAUNCH(hs_sel_hist_kernel<1>, gh, dim3(256), 0, st, a, s);
  BRP_LAUNCH(hs_sel_pick_kernel<1>, gp, dim3(64), 0, st, a, s);
  BRP_LAUNCH(hs_sel_hist_kernel<2>, gh, dim3(256), 0, st, a, s);
  BRP_LAUNCH(hs_sel_pick_kernel<2>, gp, dim3(64), 0, st, a, s);
  BRP_LAUNCH(hs_sel_emit_kernel, gh, dim3(256), 0, st, a, s);
  return launch_status();
}

}  // namespace hipk
}  // namespace brp
