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
  if (lane == leader) base = atomicAdd(counter, static_cast<uint32_t>(__popcll(mask)));
  base = __shfl(base, leader, kWave);
  if (pred) {
    const uint32_t rank = __popcll(mask & ((1ull << lane) - 1ull));
    const uint32_t slot = base + rank;
    if (slot < cap) list[slot] = make_uint2(key, __float_as_uint(power));
  }
}

// T = float (exact path) or _Float16 (config 5 spectrum); every element is
// widened to float before the reference-order float sums. Each lane gathers
// the 16 harmonics of its index straight from global memory: within a wave
// the lanes of one harmonic read at most 4l+1 consecutive words (1-3 cache
// lines), and 10 workgroups per CU keep enough gathers in flight.
// (Measured alternatives -- LDS-staged runs, XCD-contiguous tiles, 4 or 16
// indices per lane, an MFMA selection-matrix sum -- are kept out of the
// product in tools/experiments/hs_variants.hip; profiles/hs_variants_r2.txt.)
template <typename T>
__global__ void __launch_bounds__(kThreads) harmonic_sum_kernel(HSArgs a) {
#pragma clang fp contract(off)
  constexpr int TILE = kHsTile;
  static_assert(TILE % 16 == 0, "tiles start at i == 8 mod 16");
  constexpr int SPAN = TILE + kHalo;
  constexpr int SPAN_PAD = SPAN + SPAN / 16 + 1;
  __shared__ __attribute__((aligned(16))) float lds[4 * SPAN_PAD];
  float (*sv)[SPAN_PAD] = reinterpret_cast<float (*)[SPAN_PAD]>(lds);
  const int b = blockIdx.y;
  const T* P = reinterpret_cast<const T*>(sizeof(T) == 4 ? static_cast<const void*>(a.ps)
                                                        : static_cast<const void*>(a.ps16)) +
               static_cast<size_t>(b) * a.ps_stride;
  // signed: for windows below 16 the first tile starts before bin 0
  const int i0 = a.i_start + static_cast<int>(blockIdx.x) * TILE;
  const int w2 = static_cast<int>(a.w2), fhi = static_cast<int>(a.fhi), hhi = static_cast<int>(a.hhi);
  const float ninf = -__builtin_inff();
  auto ld = [&](uint32_t l, uint32_t i) -> float { return static_cast<float>(P[(l * i + 8u) >> 4]); };

  constexpr int kIt = (SPAN + kThreads - 1) / kThreads;
  float s1[kIt], s2[kIt], s3[kIt], s4[kIt], p0[kIt];
#pragma unroll
  for (int it = 0; it < kIt; ++it) {
    const int t = threadIdx.x + it * kThreads;
    const int i = i0 + t;
    s1[it] = s2[it] = s3[it] = s4[it] = ninf;
    p0[it] = 0.0f;
    if (t < SPAN && i >= w2 && i < hhi) {
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
    const int i = i0 + t;
    const bool in = t < TILE && (i >= w2 && i < fhi);
    const float p = in ? p0[it] : 0.0f;
    emit(count, list, a.cap, in && p > thr0, hs_pack(b, 0, static_cast<uint32_t>(i)), p);
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
      int j = 0;
      float m = ninf;
      if (q < ngroups) {
        const int t0 = first + q * g;
        j = (i0 + t0 + off) >> h;  // arithmetic shift: negative groups stay below w2
        if (j >= w2 && j < fhi) {
#pragma unroll
          for (int u = 0; u < 16; ++u)
            if (u < g) m = fmaxf(m, sv[h - 1][sidx(t0 + u)]);
          pred = m > thr;
        }
      }
      emit(count, list, a.cap, pred, hs_pack(b, h, static_cast<uint32_t>(j)), m);
    }
  }
}

}  // namespace

uint32_t hs_num_tiles(int32_t i_start, uint32_t hhi) {
  const int64_t span = static_cast<int64_t>(hhi) - i_start;
  if (span <= 0) return 0;
  return static_cast<uint32_t>((span + kHsTile - 1) / kHsTile);
}

hipError_t launch_harmonic_sum(const HSArgs& a, int batch, hipStream_t s) {
  const uint32_t tiles = hs_num_tiles(a.i_start, a.hhi);
  if (tiles == 0) return hipSuccess;
  const dim3 grid(tiles, batch);
  if (a.ps16 != nullptr) hipLaunchKernelGGL(harmonic_sum_kernel<_Float16>, grid, dim3(kThreads), 0, s, a);
  else hipLaunchKernelGGL(harmonic_sum_kernel<float>, grid, dim3(kThreads), 0, s, a);
  return hipGetLastError();
}

}  // namespace hipk
}  // namespace brp
