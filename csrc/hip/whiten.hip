// Whitening + RFI zapping kernels (reference demod_binary.c:857-1079, done on the
// host with FFTW/rngmed/GSL there; on MI355X it runs on the device between a
// forward and an inverse pass of the same hand-written FFT).
#include <cstdlib>

#include "hip_common.hpp"
#include "whiten_kernels.hpp"

namespace brp {
namespace hipk {

namespace {

__global__ void whiten_power_kernel(const float2* spec, uint32_t n, float* ps) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  float p = 0.0f;
  if (k != 0) {
    const float2 sk = BRP_LD(&spec[k]);
    const double re = sk.x, im = sk.y;
    p = static_cast<float>(re * re + im * im);
  }
  BRP_ST(&ps[k], p);
}

// Exact running median. Each workgroup sorts (value, position) of its span of
// SPAN inputs in LDS (bitonic; ties by position, a total order, so the order
// statistics are exactly those of the reference's sorted window) and keeps the
// inverse permutation rank[position]. Each thread owns a run of consecutive
// outputs: it finds the middle member of its first window by one scan of the
// sorted span, then slides the window one sample at a time, moving the median
// pointer past the removed / inserted ranks (O(1) members per step).
//
// CHUNKED: the first-window scan reads 8 sorted positions per 16-byte LDS
// load (the same address for every lane: a broadcast) and counts members
// branch-free, leaving the loop once every lane of the wave has found its
// median; the plain scan waits on one dependent 2-byte LDS load per entry.
// order-preserving bits of a float (any non-NaN value; -0 sorts below +0)
__device__ __forceinline__ uint32_t ord_bits(float f) {
  const uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float unord_bits(uint32_t o) {
  return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}

// REG: the span is sorted as 48-bit (ordered key, position) words, 16 per
// thread (element 16 t + j): bitonic stages with strides below 16 in
// registers, strides within a wave through cross-lane shuffles, and only the
// 3 cross-wave passes through LDS -- instead of 78 LDS passes of 2048
// compare-exchanges (which were most of the kernel's time).
template <int SPAN, int NT>
__device__ __forceinline__ void rmed_sort_reg(const float* in, uint32_t n_in, uint32_t W, uint32_t o0,
                                              uint32_t per_block, float* key, uint16_t* pos, uint16_t* rank) {
  static_assert(SPAN == 16 * NT, "16 elements per thread");
  const int t = threadIdx.x;
  uint64_t v[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int e = 16 * t + j;
    const uint32_t g = o0 + e;
    const float k = (e < static_cast<int>(per_block + W - 1) && g < n_in) ? BRP_LD(&in[g]) : __builtin_inff();
    v[j] = (static_cast<uint64_t>(ord_bits(k)) << 16) | static_cast<uint32_t>(e);
  }
  uint32_t* keyu = reinterpret_cast<uint32_t*>(key);
#pragma unroll
  for (int size = 2; size <= SPAN; size <<= 1) {
#pragma unroll
    for (int d = size >> 1; d > 0; d >>= 1) {
      if (d >= 16) {
        const int k = d >> 4;                      // partner thread t ^ k holds element e ^ d
        const bool asc = ((16 * t) & size) == 0;   // size >= 32
        const bool keep_min = ((t & k) == 0) == asc;
        if (k < kWave) {
#pragma unroll
          for (int j = 0; j < 16; ++j) {
            const uint32_t lo = __shfl_xor(static_cast<uint32_t>(v[j]), k, kWave);
            const uint32_t hi = __shfl_xor(static_cast<uint32_t>(v[j] >> 32), k, kWave);
            const uint64_t w = (static_cast<uint64_t>(hi) << 32) | lo;
            v[j] = keep_min ? (w < v[j] ? w : v[j]) : (w > v[j] ? w : v[j]);
          }
        } else {
          __syncthreads();  // the previous exchange has been read
#pragma unroll
          for (int j = 0; j < 16; ++j) {
            keyu[16 * t + j] = static_cast<uint32_t>(v[j] >> 16);
            pos[16 * t + j] = static_cast<uint16_t>(v[j]);
          }
          __syncthreads();
#pragma unroll
          for (int j = 0; j < 16; ++j) {
            const int q = (16 * t + j) ^ d;
            const uint64_t w = (static_cast<uint64_t>(keyu[q]) << 16) | pos[q];
            v[j] = keep_min ? (w < v[j] ? w : v[j]) : (w > v[j] ? w : v[j]);
          }
        }
      } else {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          if ((j & d) != 0) continue;
          const int p = j | d;
          const bool asc = ((16 * t + j) & size) == 0;
          const uint64_t a = v[j], b = v[p];
          const uint64_t mn = a < b ? a : b, mx = a < b ? b : a;
          v[j] = asc ? mn : mx;
          v[p] = asc ? mx : mn;
        }
      }
    }
  }
  __syncthreads();  // the last exchange has been read
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int e = 16 * t + j;
    key[e] = unord_bits(static_cast<uint32_t>(v[j] >> 16));
    pos[e] = static_cast<uint16_t>(v[j]);
    rank[static_cast<uint16_t>(v[j])] = static_cast<uint16_t>(e);
  }
  __syncthreads();
}

// walkers: threads that walk the window (runs of per_block / walkers outputs
// each); every walker first scans the sorted span for its first median, so
// fewer, longer runs trade that scan against the sequential walk
template <int SPAN, int NT, bool CHUNKED, bool REG = false>
__global__ void __launch_bounds__(NT) running_median_kernel(const float* in, uint32_t n_in, uint32_t W, float* med,
                                                            uint32_t n_out, uint32_t per_block, uint32_t walkers = NT) {
  __shared__ __attribute__((aligned(16))) float key[SPAN];
  __shared__ __attribute__((aligned(16))) uint16_t pos[SPAN];
  __shared__ uint16_t rank[SPAN];
  static_assert(SPAN <= 65536, "16-bit positions");
  const uint32_t o0 = blockIdx.x * per_block;
  if constexpr (REG) {
    rmed_sort_reg<SPAN, NT>(in, n_in, W, o0, per_block, key, pos, rank);
  } else {
  for (int t = threadIdx.x; t < SPAN; t += NT) {
    const uint32_t g = o0 + t;
    key[t] = (t < static_cast<int>(per_block + W - 1) && g < n_in) ? BRP_LD(&in[g]) : __builtin_inff();
    pos[t] = static_cast<uint16_t>(t);
  }
  __syncthreads();
  for (int size = 2; size <= SPAN; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = threadIdx.x; t < SPAN / 2; t += NT) {
        const int lo = 2 * t - (t & (stride - 1));
        const int hi = lo + stride;
        const bool asc = ((lo & size) == 0);
        const float ka = key[lo], kb = key[hi];
        const uint16_t pa = pos[lo], pb = pos[hi];
        const bool gt = (ka > kb) || (ka == kb && pa > pb);
        if (gt == asc) {
          key[lo] = kb;
          key[hi] = ka;
          pos[lo] = pb;
          pos[hi] = pa;
        }
      }
      __syncthreads();
    }
  }
  for (int e = threadIdx.x; e < SPAN; e += NT) rank[pos[e]] = static_cast<uint16_t>(e);
  __syncthreads();
  }

  const uint32_t mid = (W + (W & 1)) / 2 - 1;  // 0-based order statistic of the lower middle
  const bool odd = (W & 1) != 0;
  const uint32_t run = (per_block + walkers - 1) / walkers;
  const uint32_t t0 = threadIdx.x * run;
  uint32_t t1 = min(t0 + run, per_block);
  if (o0 + t1 > n_out) t1 = n_out > o0 ? n_out - o0 : 0;
  if (t0 >= t1) return;
  auto member = [&](int e, uint32_t t) {
    const uint32_t p = pos[e];
    return p >= t && p < t + W;
  };
  // first member at or after e / at or before e: 8 sorted positions per
  // 16-byte LDS load, tested branch-free (CHUNKED); one dependent 2-byte load
  // per entry otherwise. A member always exists in the searched direction.
  const uint4* pos8 = reinterpret_cast<const uint4*>(pos);
  auto members8 = [&](int c, uint32_t t) {
    const uint4 v = pos8[c];
    const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
    uint32_t mask = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint32_t p = (w4[k >> 1] >> (16 * (k & 1))) & 0xffffu;
      mask |= ((p - t) < W ? 1u : 0u) << k;  // unsigned: t <= p < t + W
    }
    return mask;
  };
  auto next_member = [&](int e, uint32_t t) {
    if constexpr (!CHUNKED) {
      while (!member(e, t)) ++e;
      return e;
    } else {
      int c = e >> 3;
      uint32_t mask = members8(c, t) & (0xffu << (e & 7));
      while (mask == 0) mask = members8(++c, t);
      return (c << 3) + __builtin_ctz(mask);
    }
  };
  auto prev_member = [&](int e, uint32_t t) {
    if constexpr (!CHUNKED) {
      while (!member(e, t)) --e;
      return e;
    } else {
      int c = e >> 3;
      uint32_t mask = members8(c, t) & (0xffu >> (7 - (e & 7)));
      while (mask == 0) mask = members8(--c, t);
      return (c << 3) + 31 - __builtin_clz(mask);
    }
  };
  // first window: scan to the mid-th member
  int m = 0;
  uint32_t below = 0;  // members with sorted index < m
  if constexpr (CHUNKED) {
    // lanes past their run (t0 >= t1) returned above; the rest scan together
    int found = -1;
    uint32_t cnt = 0;
    for (int c = 0; c < SPAN / 8; ++c) {
      const uint4 v = pos8[c];
      const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint32_t p = (w4[k >> 1] >> (16 * (k & 1))) & 0xffffu;
        const bool mem = (p - t0) < W;  // unsigned: t0 <= p < t0 + W
        if (found < 0 && mem && cnt == mid) found = c * 8 + k;
        cnt += mem ? 1u : 0u;
      }
      if (__all(found >= 0)) break;
    }
    m = found;
    below = mid;
  } else {
    for (;; ++m) {
      if (member(m, t0)) {
        if (below == mid) break;
        ++below;
      }
    }
  }
  for (uint32_t t = t0;; ++t) {
    // a = key[m]; b = next member's key (even window)
    float b = 0.0f;
    if (!odd) {
      b = key[next_member(m + 1, t)];
    }
    const float a = key[m];
    BRP_ST(&med[o0 + t], odd ? a : static_cast<float>(static_cast<double>(a + b) / 2.0));
    if (t + 1 >= t1) break;
    // slide: remove position t, insert position t + W
    const int ro = rank[t], ri = rank[t + W];
    below = below - (ro < m ? 1u : 0u) + (ri < m ? 1u : 0u);
    const uint32_t tn = t + 1;
    // restore: m is a member and exactly `mid` members lie below it
    while (below > mid) {  // move back to the previous member
      m = prev_member(m - 1, tn);
      --below;
    }
    while (!member(m, tn) || below < mid) {
      if (member(m, tn)) ++below;
      m = next_member(m + 1, tn);
    }
  }
}

// one output sample per thread; samples beyond the payload (odd n, 4-bit) are 0
__global__ void unpack_kernel(const uint8_t* packed, uint32_t n_packed, bool four_bit, double scale, float* out,
                              uint32_t n_out) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= n_out) return;
  float v = 0.0f;
  if (four_bit) {
    const uint32_t b = i >> 1;
    if (b < n_packed) {
      const uint8_t c = BRP_LD(&packed[b]);
      const uint32_t nib = (i & 1u) ? (c & 15u) : (c >> 4);
      v = static_cast<float>(static_cast<double>(static_cast<float>(nib)) / scale);
    }
  } else if (i < n_packed) {
    v = static_cast<float>(static_cast<double>(static_cast<int8_t>(BRP_LD(&packed[i]))) / scale);
  }
  BRP_ST(&out[i], v);
}

// spec[w2 + i] *= sqrt(ln2 / med[i]) for i < white_size
__global__ void whiten_scale_kernel(float2* spec, const float* med, uint32_t white_size, uint32_t w2) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= white_size) return;
  const float f = static_cast<float>(sqrt(M_LN2 / static_cast<double>(BRP_LD(&med[i]))));
  float2 v = BRP_LD(&spec[i + w2]);
  v.x *= f;
  v.y *= f;
  BRP_ST(&spec[i + w2], v);
}

__global__ void zap_kernel(float2* spec, uint32_t fft_size, const uint32_t* bins, const float2* noise, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t k = BRP_LD(&bins[i]);
  if (k < fft_size) BRP_ST(&spec[k], BRP_LD(&noise[i]));
}

// Inverse real-FFT packing: Z_k = (X_k + conj X_{M-k}) + i W_N^{-k} (X_k - conj X_{M-k}),
// with the first/last w2 bins zeroed and Im X_0 = Im X_M = 0 (FFTW c2r semantics).
__global__ void tangle_kernel(const float2* spec, uint32_t M, uint32_t fft_size, uint32_t w2, TwiddleTable tw,
                              float2* z) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= M) return;
  auto bin = [&](uint32_t q) -> float2 {
    if (q < w2 || q >= fft_size - w2) return make_float2(0.0f, 0.0f);
    float2 v = BRP_LD(&spec[q]);
    if (q == 0 || q == M) v.y = 0.0f;
    return v;
  };
  const float2 a = bin(k);
  const float2 bc = conjf2(bin(M - k));
  const float2 w = conjf2(tw_lookup32(tw, 2u * k));  // W_N^{-k}
  const float2 d = csub(a, bc);
  const float2 iwd = cmul(make_float2(0.0f, 1.0f), cmul(w, d));
  BRP_ST(&z[k], cadd(cadd(a, bc), iwd));
}

}  // namespace

hipError_t preload_whiten() {
  hipFuncAttributes at;
  return hipFuncGetAttributes(&at, reinterpret_cast<const void*>(&whiten_power_kernel));
}

hipError_t launch_unpack(const uint8_t* packed, uint32_t n_packed, bool four_bit, double scale, float* out,
                         uint32_t n_out, hipStream_t s) {
  if (n_out == 0) return hipSuccess;
  BRP_LAUNCH(unpack_kernel, dim3((n_out + 255) / 256), dim3(256), 0, s, packed, n_packed, four_bit, scale, out,
                     n_out);
  return launch_status();
}

hipError_t launch_whiten_power(const float2* spec, uint32_t n, float* ps, hipStream_t s) {
  BRP_LAUNCH(whiten_power_kernel, dim3((n + 255) / 256), dim3(256), 0, s, spec, n, ps);
  return launch_status();
}

// LDS spans: 4096 entries (32 KB) up to W = 3072, 16384 entries (128 KB, one
// workgroup per CU) up to W = 12288; wider windows: rmed_wide.hip
bool running_median_supported(uint32_t W) { return W >= 1 && W <= 12288; }

hipError_t launch_running_median(const float* in, uint32_t n_in, uint32_t W, float* med, hipStream_t s) {
  if (!running_median_supported(W) || n_in < W) return hipErrorInvalidValue;
  const uint32_t n_out = n_in - W + 1;
  if (W > 3072) {
    // 128 KB of static LDS per workgroup: gfx950 has 160 KB per CU; on a
    // device with less, the wide-window path (rmed_wide.hip) serves these W
    int dev = 0;
    int lds = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess ||
        lds < 16384 * 8)
      return hipErrorInvalidConfiguration;
    constexpr int kSpanL = 16384, kThreadsL = 1024;
    const uint32_t perL = kSpanL - W + 1;
    BRP_LAUNCH((running_median_kernel<kSpanL, kThreadsL, true>), dim3((n_out + perL - 1) / perL),
                       dim3(kThreadsL), 0, s, in, n_in, W, med, n_out, perL);
    return launch_status();
  }
  constexpr int kSpan = 4096, kThreads = 256;
  const uint32_t per = kSpan - W + 1;
  static const bool plain = std::getenv("BRP_RMED_PLAIN") != nullptr;  // A/B switch
  static const int walkers_env = std::getenv("BRP_RMED_WALKERS") ? std::atoi(std::getenv("BRP_RMED_WALKERS")) : 0;
  const uint32_t walkers = static_cast<uint32_t>(walkers_env > 0 ? std::min(kThreads, walkers_env) : kThreads);
  // register/shuffle sort by default (655 -> 503 us per whitening median on
  // MI355X, bit-exact; profiles/README.md round 3); BRP_RMED_REG=0: LDS bitonic
  static const bool reg = std::getenv("BRP_RMED_REG") == nullptr || std::atoi(std::getenv("BRP_RMED_REG")) != 0;
  if (reg && !plain)
    BRP_LAUNCH((running_median_kernel<kSpan, kThreads, true, true>), dim3((n_out + per - 1) / per),
                       dim3(kThreads), 0, s, in, n_in, W, med, n_out, per, walkers);
  else if (plain)
    BRP_LAUNCH((running_median_kernel<kSpan, kThreads, false>), dim3((n_out + per - 1) / per), dim3(kThreads), 0,
                       s, in, n_in, W, med, n_out, per);
  else
    BRP_LAUNCH((running_median_kernel<kSpan, kThreads, true>), dim3((n_out + per - 1) / per), dim3(kThreads), 0,
                       s, in, n_in, W, med, n_out, per);
  return launch_status();
}

hipError_t launch_whiten_scale(float2* spec, const float* med, uint32_t white_size, uint32_t w2, hipStream_t s) {
  BRP_LAUNCH(whiten_scale_kernel, dim3((white_size + 255) / 256), dim3(256), 0, s, spec, med, white_size, w2);
  return launch_status();
}

hipError_t launch_zap(float2* spec, uint32_t fft_size, const uint32_t* bins, const float2* noise, uint32_t n,
                      hipStream_t s) {
  if (n == 0) return hipSuccess;
  BRP_LAUNCH(zap_kernel, dim3((n + 255) / 256), dim3(256), 0, s, spec, fft_size, bins, noise, n);
  return launch_status();
}

hipError_t launch_tangle(const float2* spec, uint32_t M, uint32_t fft_size, uint32_t w2, const TwiddleTable& tw,
                         float2* z, hipStream_t s) {
  BRP_LAUNCH(tangle_kernel, dim3((M + 255) / 256), dim3(256), 0, s, spec, M, fft_size, w2, tw, z);
  return launch_status();
}

}  // namespace hipk
}  // namespace brp
