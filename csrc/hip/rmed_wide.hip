// Exact running median for wide windows (W > 3072, up to the reference's
// 250 000, demod_binary.c:245-263; rngmed.c:48-341 computes it on the host).
//
// The LDS kernel of whiten.hip sorts each workgroup's span (outputs + W - 1
// inputs <= 4096) in LDS; a wide window does not fit. Here the whole input is
// sorted ONCE (stable LSD radix sort of the float keys carrying positions:
// ties stay in position order, a total order, so the order statistics are
// exactly the reference's), giving sp[e] = position of the e-th smallest and
// rank[p] = e. The median of window [t, t+W) is then the element of the
// mid-th smallest rank among rank[t .. t+W-1]:
//   * one wave per run of consecutive outputs finds its first window's median
//     rank by a radix select over those W ranks (LDS histogram per 8-bit
//     digit, one coalesced pass over the window per digit);
//   * it then slides: removing rank[t] and inserting rank[t+W] moves the
//     median pointer m (a sorted index) by O(1) members; the next / previous
//     member (t <= sp[e] < t + W) is found 256 sorted entries per probe with
//     a ballot over the wave.
// Even windows average the two middle members in the reference's arithmetic.
#include <cstdint>

#include "hip_common.hpp"
#include "whiten_kernels.hpp"

namespace brp {
namespace hipk {

namespace {

constexpr int kRsThreads = 256;
constexpr int kRsPer = 16;
constexpr int kRsTile = kRsThreads * kRsPer;  // elements per radix-sort block
constexpr uint32_t kRmedRun = 4096;            // outputs per wave

// order-preserving float -> uint (-0 folds onto +0: equal values, position order)
__device__ __forceinline__ uint32_t sort_key(float f) {
  uint32_t u = __float_as_uint(f);
  if (u == 0x80000000u) u = 0;
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__global__ void __launch_bounds__(kRsThreads) rs_init(const float* in, uint32_t n, uint32_t* keys, uint32_t* vals) {
  const uint32_t i = blockIdx.x * kRsThreads + threadIdx.x;
  if (i >= n) return;
  BRP_ST(&keys[i], sort_key(BRP_LD(&in[i])));
  BRP_ST(&vals[i], i);
}

// digit histogram of one tile; hist is digit-major: hist[d * nblocks + block]
__global__ void __launch_bounds__(kRsThreads) rs_hist(const uint32_t* keys, uint32_t n, int shift, uint32_t* hist,
                                                      uint32_t nblocks) {
  __shared__ uint32_t h[256];
  h[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t b0 = blockIdx.x * kRsTile;
#pragma unroll 4
  for (int r = 0; r < kRsPer; ++r) {
    const uint32_t i = b0 + r * kRsThreads + threadIdx.x;
    if (i < n) atomicAdd(&h[(BRP_LD(&keys[i]) >> shift) & 255u], 1u);
  }
  __syncthreads();
  BRP_ST(&hist[threadIdx.x * nblocks + blockIdx.x], h[threadIdx.x]);
}

// exclusive scan of hist[0 .. total) in place, one workgroup
__global__ void __launch_bounds__(1024) rs_scan(uint32_t* hist, uint32_t total) {
  __shared__ uint32_t part[1024];
  const uint32_t per = (total + 1023) / 1024;
  const uint32_t lo = threadIdx.x * per, hi = min(lo + per, total);
  uint32_t s = 0;
  for (uint32_t i = lo; i < hi; ++i) s += BRP_LD(&hist[i]);
  part[threadIdx.x] = s;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    const uint32_t v = threadIdx.x >= static_cast<uint32_t>(off) ? part[threadIdx.x - off] : 0u;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  uint32_t run = threadIdx.x ? part[threadIdx.x - 1] : 0u;
  for (uint32_t i = lo; i < hi; ++i) {
    const uint32_t c = BRP_LD(&hist[i]);
    BRP_ST(&hist[i], run);
    run += c;
  }
}

// stable scatter of one tile: element r*256 + t of the tile is processed in
// round r by thread t, so tile order == (round, thread) order; ranks within a
// round come from a ballot match on the 8 digit bits and per-wave counts
__global__ void __launch_bounds__(kRsThreads) rs_scatter(const uint32_t* kin, const uint32_t* vin, uint32_t* kout,
                                                         uint32_t* vout, uint32_t n, int shift, const uint32_t* offs,
                                                         uint32_t nblocks) {
  constexpr int kWaves = kRsThreads / kWave;
  __shared__ uint32_t base[256];
  __shared__ uint32_t wcnt[kWaves][256];
  base[threadIdx.x] = BRP_LD(&offs[threadIdx.x * nblocks + blockIdx.x]);
#pragma unroll
  for (int w = 0; w < kWaves; ++w) wcnt[w][threadIdx.x] = 0;
  __syncthreads();
  const int lane = threadIdx.x % kWave, wave = threadIdx.x / kWave;
  const unsigned long long lt = (1ull << lane) - 1ull;
  const uint32_t b0 = blockIdx.x * kRsTile;
  for (int r = 0; r < kRsPer; ++r) {
    const uint32_t i = b0 + r * kRsThreads + threadIdx.x;
    const bool valid = i < n;
    const uint32_t k = valid ? BRP_LD(&kin[i]) : 0u;
    const uint32_t v = valid ? BRP_LD(&vin[i]) : 0u;
    const uint32_t d = (k >> shift) & 255u;
    unsigned long long same = __ballot(valid);
#pragma unroll
    for (int bit = 0; bit < 8; ++bit) {
      const bool set = (d >> bit) & 1u;
      const unsigned long long bb = __ballot(set);
      same &= set ? bb : ~bb;
    }
    const uint32_t rw = __popcll(same & lt);
    if (valid && rw == 0) wcnt[wave][d] = __popcll(same);
    __syncthreads();
    if (valid) {
      uint32_t pre = 0;
      for (int w = 0; w < wave; ++w) pre += wcnt[w][d];
      const uint32_t pos = base[d] + pre + rw;
      BRP_ST(&kout[pos], k);
      BRP_ST(&vout[pos], v);
    }
    __syncthreads();
    uint32_t add = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) {
      add += wcnt[w][threadIdx.x];
      wcnt[w][threadIdx.x] = 0;
    }
    base[threadIdx.x] += add;
    __syncthreads();
  }
}

__global__ void __launch_bounds__(kRsThreads) rs_rank(const uint32_t* sp, uint32_t n, uint32_t* rank) {
  const uint32_t e = blockIdx.x * kRsThreads + threadIdx.x;
  if (e < n) BRP_ST(&rank[BRP_LD(&sp[e])], e);
}

// one wave per run of kRmedRun outputs
__global__ void __launch_bounds__(kWave) rmed_wide_kernel(const float* in, uint32_t n_in, uint32_t W, const uint32_t* sp,
                                                          const uint32_t* rank, float* med, uint32_t n_out, int nbits) {
  __shared__ uint32_t hist[256];
  const uint32_t t0 = blockIdx.x * kRmedRun;
  if (t0 >= n_out) return;
  const uint32_t t1 = min(t0 + kRmedRun, n_out);
  const int lane = threadIdx.x;
  const uint32_t mid = (W + (W & 1u)) / 2 - 1;  // 0-based order statistic of the lower middle
  const bool odd = (W & 1u) != 0;

  // radix select of the mid-th smallest rank in [t0, t0 + W), top digit first
  uint32_t prefix = 0, k = mid;
  int done_bits = 0;
  while (done_bits < nbits) {
    const int width = min(8, nbits - done_bits);
    const int shift = nbits - done_bits - width;
#pragma unroll
    for (int q = 0; q < 4; ++q) hist[lane + 64 * q] = 0;
    __syncthreads();
    for (uint32_t p = t0 + lane; p < t0 + W; p += kWave) {
      const uint32_t r = BRP_LD(&rank[p]);
      if ((static_cast<uint64_t>(r) >> (shift + width)) == prefix) atomicAdd(&hist[(r >> shift) & ((1u << width) - 1u)], 1u);
    }
    __syncthreads();
    // lane owns bins 4 lane .. 4 lane + 3; inclusive scan across lanes
    uint32_t c[4], s = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      c[q] = hist[4 * lane + q];
      s += c[q];
    }
    uint32_t incl = s;
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
      const uint32_t v = __shfl_up(incl, off, kWave);
      if (lane >= off) incl += v;
    }
    uint32_t below = incl - s;  // counts of bins before this lane's first bin
    int dsel = -1;
    uint32_t kk = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (dsel < 0 && k < below + c[q]) {
        dsel = 4 * lane + q;
        kk = k - below;
      }
      below += c[q];
    }
    const unsigned long long hit = __ballot(dsel >= 0);
    const int src = __ffsll(static_cast<long long>(hit)) - 1;
    const int d = __shfl(dsel, src, kWave);
    k = __shfl(kk, src, kWave);
    prefix = (prefix << width) | static_cast<uint32_t>(d);
    done_bits += width;
    __syncthreads();
  }
  uint32_t m = prefix;     // sorted index of the median member of window t0
  uint32_t below = mid;    // members with sorted index < m

  auto is_member = [&](uint32_t e, uint32_t t) -> bool {
    const uint32_t p = BRP_LD(&sp[e]);
    return (p - t) < W;
  };
  // first member with sorted index >= e (exists: the window has W members)
  // (bounded: past the end it returns n_in - 1, so a broken invariant gives a
  // wrong value, never a hung wave)
  auto next_member = [&](uint32_t e, uint32_t t) -> uint32_t {
    for (; e < n_in; e += 4 * kWave) {
      bool f[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t x = e + lane + kWave * q;
        f[q] = x < n_in && ((BRP_LD(&sp[x]) - t) < W);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const unsigned long long b = __ballot(f[q]);
        if (b) return e + kWave * q + (__ffsll(static_cast<long long>(b)) - 1);
      }
    }
    return n_in - 1;
  };
  // last member with sorted index <= e
  auto prev_member = [&](uint32_t e, uint32_t t) -> uint32_t {
    for (;; e -= 4 * kWave) {
      bool f[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t off = static_cast<uint32_t>(lane + kWave * q);
        f[q] = off <= e && ((BRP_LD(&sp[e - off]) - t) < W);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const unsigned long long b = __ballot(f[q]);
        if (b) return e - (kWave * q + (__ffsll(static_cast<long long>(b)) - 1));
      }
      if (e < 4 * kWave) return 0;
    }
  };

  uint32_t ro_v = 0, ri_v = 0;
  for (uint32_t t = t0;; ++t) {
    const uint32_t step = t - t0;
    if (step % kWave == 0) {
      // ranks leaving / entering over the next 64 slides
      const uint32_t po = t + lane, pi = t + W + lane;
      ro_v = po < n_in ? BRP_LD(&rank[po]) : 0u;
      ri_v = pi < n_in ? BRP_LD(&rank[pi]) : 0u;
    }
    const float a = BRP_LD(&in[BRP_LD(&sp[m])]);
    float out;
    if (odd) {
      out = a;
    } else {
      const float b = BRP_LD(&in[BRP_LD(&sp[next_member(m + 1, t)])]);
      out = static_cast<float>(static_cast<double>(a + b) / 2.0);
    }
    if (lane == 0) BRP_ST(&med[t], out);
    if (t + 1 >= t1) break;
    const uint32_t ro = __shfl(ro_v, static_cast<int>(step % kWave), kWave);
    const uint32_t ri = __shfl(ri_v, static_cast<int>(step % kWave), kWave);
    below = below - (ro < m ? 1u : 0u) + (ri < m ? 1u : 0u);
    const uint32_t tn = t + 1;
    // restore: m is a member and exactly `mid` members lie below it
    while (below > mid) {
      m = prev_member(m - 1, tn);
      --below;
    }
    for (uint32_t guard = 0; guard < W; ++guard) {
      const bool mem = is_member(m, tn);
      if (mem && below >= mid) break;
      if (mem) ++below;
      m = next_member(m + 1, tn);
    }
  }
}

int bits_for(uint32_t n) {
  int b = 1;
  while (b < 32 && (1ull << b) < n) ++b;
  return b;
}

}  // namespace

size_t running_median_wide_scratch_bytes(uint32_t n_in) {
  const size_t nblocks = (n_in + kRsTile - 1) / kRsTile;
  return sizeof(uint32_t) * (5ull * n_in + 256ull * nblocks + 64);
}

hipError_t preload_rmed_wide() {
  hipFuncAttributes at;
  return hipFuncGetAttributes(&at, reinterpret_cast<const void*>(&rs_init));
}

hipError_t launch_running_median_wide(const float* in, uint32_t n_in, uint32_t W, float* med, void* scratch,
                                      hipStream_t s) {
  if (W == 0 || n_in < W || scratch == nullptr) return hipErrorInvalidValue;
  const uint32_t n_out = n_in - W + 1;
  const uint32_t nblocks = (n_in + kRsTile - 1) / kRsTile;
  uint32_t* base = static_cast<uint32_t*>(scratch);
  uint32_t* keys[2] = {base, base + n_in};
  uint32_t* vals[2] = {base + 2ull * n_in, base + 3ull * n_in};
  uint32_t* rank = base + 4ull * n_in;
  uint32_t* hist = base + 5ull * n_in;
  const dim3 eg((n_in + kRsThreads - 1) / kRsThreads);
  BRP_LAUNCH(rs_init, eg, dim3(kRsThreads), 0, s, in, n_in, keys[0], vals[0]);
  for (int pass = 0; pass < 4; ++pass) {
    const int src = pass & 1, dst = src ^ 1;
    BRP_LAUNCH(rs_hist, dim3(nblocks), dim3(kRsThreads), 0, s, keys[src], n_in, 8 * pass, hist, nblocks);
    BRP_LAUNCH(rs_scan, dim3(1), dim3(1024), 0, s, hist, 256u * nblocks);
    BRP_LAUNCH(rs_scatter, dim3(nblocks), dim3(kRsThreads), 0, s, keys[src], vals[src], keys[dst], vals[dst],
                       n_in, 8 * pass, hist, nblocks);
  }
  // four passes: the sorted positions are back in vals[0]
  BRP_LAUNCH(rs_rank, eg, dim3(kRsThreads), 0, s, vals[0], n_in, rank);
  const dim3 rg((n_out + kRmedRun - 1) / kRmedRun);
  BRP_LAUNCH(rmed_wide_kernel, rg, dim3(kWave), 0, s, in, n_in, W, vals[0], rank, med, n_out, bits_for(n_in));
  return launch_status();
}

}  // namespace hipk
}  // namespace brp
