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

#include "hip_common.hpp"
#include "hs_kernels.hpp"

namespace brp {
namespace hipk {

namespace {

constexpr int kThreads = 256;
constexpr int kHalo = 4;
constexpr int kSpan = kHsTile + kHalo;
constexpr int kSpanPad = kSpan + kSpan / 16 + 1;
__device__ __forceinline__ int sidx(int t) { return t + (t >> 4); }

__device__ __forceinline__ void emit(uint32_t* counter, uint2* list, uint32_t cap, bool pred, uint32_t key,
                                     float power) {
  const unsigned long long mask = __ballot(pred);
  if (mask == 0) return;
  const int lane = threadIdx.x % kWave;
  const int leader = __ffsll(static_cast<long long>(mask)) - 1;
  uint32_t base = 0;
  if (lane == leader) base = atomicAdd(counter, static_cast<uint32_t>(__popcll(mask)));
  base = __shfl(base, leader, kWave);
  if (pred) {
    const uint32_t rank = __popcll(mask & ((1ull << lane) - 1ull));
    const uint32_t slot = base + rank;
    if (slot < cap) list[slot] = make_uint2(key, __float_as_uint(power));
  }
}

// LDS staging of the harmonic segments: for harmonic l the tile's bins
// (l*i + 8) >> 4, i in [i0, i0 + kSpan), form one contiguous run of about
// l*kSpan/16 bins. All 16 runs (8.5 bins per i in total) are copied into LDS
// with 16-B loads, so the 16 per-i gathers become LDS reads (conflict free:
// the lanes of a wave read at most 4l consecutive words). The run of harmonic
// l starts at the 4-aligned bin lo4(l) and occupies kStageCap(l) floats.
__host__ __device__ constexpr int stage_cap(int l) { return ((l * (kSpan - 1) / 16 + 5 + 3) / 4) * 4; }
__host__ __device__ constexpr int stage_off(int l) { return l <= 1 ? 0 : stage_off(l - 1) + stage_cap(l - 1); }
// per harmonic l: ceil(chunks / threads) load iterations
__host__ __device__ constexpr int stage_iters(int l) { return (stage_cap(l) / 4 + kThreads - 1) / kThreads; }
__host__ __device__ constexpr int stage_iters_before(int l) { return l <= 1 ? 0 : stage_iters_before(l - 1) + stage_iters(l - 1); }
// LDS floats of the kernel staging harmonics 1..smax (S_1..S_4 alias the area)
__host__ __device__ constexpr int stage_lds_floats(int smax) {
  return stage_off(smax + 1) > 4 * kSpanPad ? stage_off(smax + 1) : 4 * kSpanPad;
}

// f(integral_constant<l>, integral_constant<it>, flat iteration base) for
// l = 1..LMAX and it < stage_iters(l), fully unrolled
template <int LMAX, int L, int IT, typename F>
__device__ __forceinline__ void stage_for_each_impl(F&& f) {
  if constexpr (L <= LMAX) {
    if constexpr (IT < stage_iters(L)) {
      f(std::integral_constant<int, L>{}, std::integral_constant<int, IT>{}, stage_iters_before(L));
      stage_for_each_impl<LMAX, L, IT + 1>(f);
    } else {
      stage_for_each_impl<LMAX, L + 1, 0>(f);
    }
  }
}
template <int LMAX, typename F>
__device__ __forceinline__ void stage_for_each(F&& f) {
  stage_for_each_impl<LMAX, 1, 0>(f);
}

// T = float (exact path) or _Float16 (config 5 spectrum); every element is
// widened to float before the reference-order float sums. Harmonics 1..SMAX
// are staged in LDS (their runs are short, l/16 bins per i, and shared by
// many lanes of a gather), harmonics SMAX+1..16 are gathered per i from
// global memory: SMAX = 0 gathers all, 16 stages all.
template <typename T, int SMAX, int TILE>
__global__ void __launch_bounds__(kThreads) harmonic_sum_kernel(HSArgs a) {
#pragma clang fp contract(off)
  constexpr bool STAGED = SMAX > 0;
  static_assert(!STAGED || TILE == kHsTile, "LDS staging is laid out for the default tile");
  static_assert(TILE % 16 == 0, "tiles start at i == 8 mod 16");
  constexpr int SPAN = TILE + kHalo;
  constexpr int SPAN_PAD = SPAN + SPAN / 16 + 1;
  // staged segments, then (after a barrier) S_1..S_4 over the tile + halo
  __shared__ __attribute__((aligned(16))) float lds[STAGED ? stage_lds_floats(SMAX) : 4 * SPAN_PAD];
  float (*sv)[SPAN_PAD] = reinterpret_cast<float (*)[SPAN_PAD]>(lds);
  const int b = blockIdx.y;
  const T* P = reinterpret_cast<const T*>(sizeof(T) == 4 ? static_cast<const void*>(a.ps)
                                                        : static_cast<const void*>(a.ps16)) +
               static_cast<size_t>(b) * a.ps_stride;
  const uint32_t tile_id = a.xcd != 0 ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
  const uint32_t i0 = a.i_start + tile_id * TILE;
  const float ninf = -__builtin_inff();
  auto lo4 = [&](uint32_t l) { return ((l * i0 + 8u) >> 4) & ~3u; };

  if constexpr (STAGED) {
    // harmonic by harmonic (compile-time l: the run's origin is a scalar and
    // no per-lane selection is needed); every load is issued before the first
    // LDS write. Chunks past the spectrum's stride read as zero (only i >= hhi
    // would use them).
    constexpr int kIters = stage_iters_before(SMAX + 1);
    float4 v[kIters];
    stage_for_each<SMAX>([&](auto l_tag, auto it_tag, int it_base) {
      constexpr int l = decltype(l_tag)::value;
      constexpr int it = decltype(it_tag)::value;
      constexpr int nch = stage_cap(l) / 4;
      const int ch = static_cast<int>(threadIdx.x) + it * kThreads;
      v[it_base + it] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (ch < nch) {
        const uint32_t bin = lo4(l) + 4u * static_cast<uint32_t>(ch);
        if (bin + 4 <= a.ps_stride) {
          if constexpr (sizeof(T) == 4) {
            v[it_base + it] = *reinterpret_cast<const float4*>(P + bin);
          } else {
            const uint2 h = *reinterpret_cast<const uint2*>(P + bin);
            const _Float16* hh = reinterpret_cast<const _Float16*>(&h);
            v[it_base + it] = make_float4(static_cast<float>(hh[0]), static_cast<float>(hh[1]),
                                          static_cast<float>(hh[2]), static_cast<float>(hh[3]));
          }
        }
      }
    });
    stage_for_each<SMAX>([&](auto l_tag, auto it_tag, int it_base) {
      constexpr int l = decltype(l_tag)::value;
      constexpr int it = decltype(it_tag)::value;
      const int ch = static_cast<int>(threadIdx.x) + it * kThreads;
      if (ch < stage_cap(l) / 4) reinterpret_cast<float4*>(lds + stage_off(l))[ch] = v[it_base + it];
    });
    __syncthreads();
  }
  auto ld = [&](uint32_t l, uint32_t i) -> float {
    const uint32_t bin = (l * i + 8u) >> 4;
    if (static_cast<int>(l) <= SMAX) return lds[stage_off(static_cast<int>(l)) + static_cast<int>(bin - lo4(l))];
    return static_cast<float>(P[bin]);
  };

  constexpr int kIt = (SPAN + kThreads - 1) / kThreads;
  float s1[kIt], s2[kIt], s3[kIt], s4[kIt], p0[kIt];
#pragma unroll
  for (int it = 0; it < kIt; ++it) {
    const int t = threadIdx.x + it * kThreads;
    const uint32_t i = i0 + t;
    s1[it] = s2[it] = s3[it] = s4[it] = ninf;
    p0[it] = 0.0f;
    if (t < SPAN && i >= a.w2 && i < a.hhi) {
      float sum = ld(16, i);
      p0[it] = sum;
      sum += ld(8, i);
      s1[it] = sum;
      sum += ld(12, i) + ld(4, i);
      s2[it] = sum;
      sum += ld(14, i) + ld(10, i) + ld(6, i) + ld(2, i);
      s3[it] = sum;
      sum += ld(15, i) + ld(13, i) + ld(11, i) + ld(9, i) + ld(7, i) + ld(5, i) + ld(3, i) + ld(1, i);
      s4[it] = sum;
    }
  }
  if constexpr (STAGED) __syncthreads();  // staging area becomes sv
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
  const float thr0 = a.thr[static_cast<size_t>(b) * kHsThrStride + 0];
  // level 0: the power spectrum itself (kept in registers from the S_1 sums)
#pragma unroll
  for (int it = 0; it < kIt; ++it) {
    const int t = threadIdx.x + it * kThreads;
    if (t - static_cast<int>(threadIdx.x) >= TILE) break;  // uniform: whole iterations past the tile
    const uint32_t i = i0 + t;
    const bool in = t < TILE && (i >= a.w2 && i < a.fhi);
    const float p = in ? p0[it] : 0.0f;
    emit(count, list, a.cap, in && p > thr0, hs_pack(b, 0, i), p);
  }
  // levels 1..4: group of 2^h consecutive i starting at s == 2^(h-1) mod 2^h;
  // one thread per group, stride-2^h reads made (nearly) conflict free by the
  // t + t/16 padding of sv
#pragma unroll
  for (int h = 1; h <= 4; ++h) {
    const int g = 1 << h;
    const int off = g >> 1;
    const float thr = a.thr[static_cast<size_t>(b) * kHsThrStride + h];
    const int first = static_cast<int>((off - (i0 % g) + g) % g);
    const int ngroups = (TILE - first + g - 1) / g;
    for (int q = threadIdx.x; q < ((ngroups + kThreads - 1) / kThreads) * kThreads; q += kThreads) {
      bool pred = false;
      uint32_t j = 0;
      float m = ninf;
      if (q < ngroups) {
        const int t0 = first + q * g;
        j = (i0 + static_cast<uint32_t>(t0) + off) >> h;
        if (j >= a.w2 && j < a.fhi) {
#pragma unroll
          for (int u = 0; u < 16; ++u)
            if (u < g) m = fmaxf(m, sv[h - 1][sidx(t0 + u)]);
          pred = m > thr;
        }
      }
      emit(count, list, a.cap, pred, hs_pack(b, h, j), m);
    }
  }
}

}  // namespace

uint32_t hs_num_tiles(uint32_t i_start, uint32_t hhi, uint32_t tile) {
  if (hhi <= i_start) return 0;
  return (hhi - i_start + tile - 1) / tile;
}

hipError_t launch_harmonic_sum(const HSArgs& a, int batch, hipStream_t s) {
  const uint32_t tile = a.tile != 0 ? a.tile : kHsTile;
  if (a.staged_harmonics != 0 && tile != kHsTile) return hipErrorInvalidValue;
  const uint32_t tiles = hs_num_tiles(a.i_start, a.hhi, tile);
  if (tiles == 0) return hipSuccess;
  const dim3 grid(tiles, batch);
#define BRP_HS_LAUNCH(SM, TL)                                                                                   \
  if (a.ps16 != nullptr) hipLaunchKernelGGL((harmonic_sum_kernel<_Float16, SM, TL>), grid, dim3(kThreads), 0, s, a); \
  else hipLaunchKernelGGL((harmonic_sum_kernel<float, SM, TL>), grid, dim3(kThreads), 0, s, a);
  switch (a.staged_harmonics) {
    case 0:
      switch (tile) {
        case kHsTile: BRP_HS_LAUNCH(0, kHsTile) break;
        case 1008: BRP_HS_LAUNCH(0, 1008) break;
        case 2032: BRP_HS_LAUNCH(0, 2032) break;
        case 496: BRP_HS_LAUNCH(0, 496) break;
        default: return hipErrorInvalidValue;
      }
      break;
    case 4: BRP_HS_LAUNCH(4, kHsTile) break;
    case 8: BRP_HS_LAUNCH(8, kHsTile) break;
    case 16: BRP_HS_LAUNCH(16, kHsTile) break;
    default: return hipErrorInvalidValue;
  }
#undef BRP_HS_LAUNCH
  return hipGetLastError();
}

}  // namespace hipk
}  // namespace brp
