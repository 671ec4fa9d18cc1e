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

// MODE HS_F32: fp32 spectrum (exact path). HS_F16: fp16 spectrum (config 5),
// widened to float before the reference-order float sums.
//
// Each lane gathers the 16 harmonics of its index straight from global memory:
// within a wave the lanes of one harmonic read at most 4l+1 consecutive words
// (1-3 cache lines), and 10 workgroups per CU keep enough gathers in flight.
// (Measured alternatives -- LDS-staged runs, XCD-contiguous tiles, 4 or 16
// indices per lane, an MFMA selection-matrix sum -- are kept out of the
// product in tools/experiments/hs_variants.hip; profiles/hs_variants_r2.txt.)
template <int MODE>
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
  switch (a.mode) {
    case HS_F16: hipLaunchKernelGGL(harmonic_sum_kernel<HS_F16>, grid, dim3(kThreads), 0, s, a); break;
    default: hipLaunchKernelGGL(harmonic_sum_kernel<HS_F32>, grid, dim3(kThreads), 0, s, a); break;
  }
  return hipGetLastError();
}

}  // namespace hipk
}  // namespace brp
