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

// T = float (exact path) or _Float16 (config 5 spectrum); every element is
// widened to float before the reference-order float sums
template <typename T>
__global__ void __launch_bounds__(kThreads) harmonic_sum_kernel(HSArgs a) {
#pragma clang fp contract(off)
  __shared__ __attribute__((aligned(16))) float sv[4][kSpanPad];  // S_1..S_4 over the tile + halo
  const int b = blockIdx.y;
  const T* P = reinterpret_cast<const T*>(sizeof(T) == 4 ? static_cast<const void*>(a.ps)
                                                        : static_cast<const void*>(a.ps16)) +
               static_cast<size_t>(b) * a.ps_stride;
  auto ld = [&](uint32_t idx) { return static_cast<float>(P[idx]); };
  const uint32_t i0 = a.i_start + blockIdx.x * kHsTile;
  const float ninf = -__builtin_inff();

  for (int t = threadIdx.x; t < kSpan; t += kThreads) {
    const uint32_t i = i0 + t;
    float s1 = ninf, s2 = ninf, s3 = ninf, s4 = ninf;
    if (i >= a.w2 && i < a.hhi) {
      float sum = ld(i);
      sum += ld((8u * i + 8u) >> 4);
      s1 = sum;
      sum += ld((12u * i + 8u) >> 4) + ld((4u * i + 8u) >> 4);
      s2 = sum;
      sum += ld((14u * i + 8u) >> 4) + ld((10u * i + 8u) >> 4) + ld((6u * i + 8u) >> 4) + ld((2u * i + 8u) >> 4);
      s3 = sum;
      sum += ld((15u * i + 8u) >> 4) + ld((13u * i + 8u) >> 4) + ld((11u * i + 8u) >> 4) + ld((9u * i + 8u) >> 4) +
             ld((7u * i + 8u) >> 4) + ld((5u * i + 8u) >> 4) + ld((3u * i + 8u) >> 4) + ld((i + 8u) >> 4);
      s4 = sum;
    }
    sv[0][sidx(t)] = s1;
    sv[1][sidx(t)] = s2;
    sv[2][sidx(t)] = s3;
    sv[3][sidx(t)] = s4;
  }
  __syncthreads();

  uint32_t* count = &a.list[0].x;
  uint2* list = a.list + 1;
  const float thr0 = a.thr[static_cast<size_t>(b) * kHsThrStride + 0];
  // level 0: the power spectrum itself
  for (int t = threadIdx.x; t < kHsTile; t += kThreads) {
    const uint32_t i = i0 + t;
    const bool in = (i >= a.w2 && i < a.fhi);
    const float p = in ? ld(i) : 0.0f;
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
    const int ngroups = (kHsTile - first + g - 1) / g;
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

uint32_t hs_num_tiles(uint32_t i_start, uint32_t hhi) {
  if (hhi <= i_start) return 0;
  return (hhi - i_start + kHsTile - 1) / kHsTile;
}

hipError_t launch_harmonic_sum(const HSArgs& a, int batch, hipStream_t s) {
  const uint32_t tiles = hs_num_tiles(a.i_start, a.hhi);
  if (tiles == 0) return hipSuccess;
  if (a.ps16 != nullptr)
    hipLaunchKernelGGL(harmonic_sum_kernel<_Float16>, dim3(tiles, batch), dim3(kThreads), 0, s, a);
  else
    hipLaunchKernelGGL(harmonic_sum_kernel<float>, dim3(tiles, batch), dim3(kThreads), 0, s, a);
  return hipGetLastError();
}

}  // namespace hipk
}  // namespace brp
