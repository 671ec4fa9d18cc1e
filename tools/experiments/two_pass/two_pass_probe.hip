// Memory-shape probe of a two-pass packed FFT for the benchmark plan
// (M = 24576 x 256 complex), not part of the product.
//
// Today's three passes move, per template, 17 MB (series gather) + 50 MB
// (pass 1 write) + 100 MB (pass 2 in place) + 50 MB (pass 3 read) + 21 MB
// (spectrum). The two-pass shape fuses passes 1 and 2 into one column
// transform of 24576 points per n3 (one workgroup per column, register/LDS
// resident), written transposed ([n3][c], contiguous), and reads pass 3's
// rows as [n3][16 rows] tiles:
//   A : gather 8192 complex (the non-padding third) at stride 256 complex,
//       3 x 3 LDS round trips of 64 KB (the FFT's exchanges), write 24576
//       complex contiguous                                   (17 + 50 MB)
//   A0: A without the LDS round trips (gather + write only); A_conflict_free_R:
//       R round trips per set with lane-consecutive (conflict-free) addresses
//   B : 16 rows + their 16 mirror rows per workgroup read as 2 x 256 pieces
//       of 128 B, powers written as 64-B pieces of bins c + C k3 (50 + 21 MB)
//   P1/P2/P3: today's passes as memory shapes (16-column gather + write;
//       16-column tiles in place; 8-row pairs read + 32-B pieces out)
// Every kernel runs T = 3 templates in one launch (the three pipelines).
// Build: hipcc --offload-arch=gfx950 -O3 -o build/probe/two_pass_probe tools/experiments/two_pass_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CHECK(x)                                                                     \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) {                                                           \
      std::printf("HIP error %s at line %d\n", hipGetErrorName(e), __LINE__);        \
      return 1;                                                                      \
    }                                                                                \
  } while (0)

constexpr uint32_t L1 = 192, L2 = 128, L3 = 256, C = L1 * L2, M = C * L3;
constexpr uint32_t NNZ = C / 3;          // non-padding inputs of a column
constexpr uint32_t LIMIT = 5272839;      // spectrum bins written
constexpr uint32_t T = 3;                // templates per launch
constexpr uint32_t NSER = 1u << 22;      // series samples

__device__ __forceinline__ uint32_t xcd_col(uint32_t b, uint32_t n) {
  // blocks b, b+8, ... run on one XCD: give each XCD a contiguous column range
  return (b % 8) * (n / 8) + b / 8;
}

template <bool LDS, int ROUNDS = 3, bool CONFLICT = true>
__global__ void __launch_bounds__(1024) passA(const float* __restrict__ ser, float2* __restrict__ out) {
  __shared__ float2 lds[8192];
  const uint32_t n3 = xcd_col(blockIdx.x, L3);
  const uint32_t t = threadIdx.x;
  float2 v[24];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t np = t + 1024 * j;  // n' = n1 * 128 + n2
    const uint32_t n = (np >> 7) * (L2 * L3) + (np & 127) * L3 + n3;
    const uint32_t m = (2 * n + 17 * blockIdx.y) & (NSER - 2);
    v[j] = make_float2(ser[m], ser[m + 1]);
  }
#pragma unroll
  for (int j = 8; j < 24; ++j) v[j] = make_float2(v[j - 8].y, v[j - 8].x + 1.0f);
  if constexpr (LDS) {
    for (int s = 0; s < 3; ++s) {
#pragma unroll
      for (int r = 0; r < ROUNDS; ++r) {
#pragma unroll
        for (int j = 0; j < 8; ++j) lds[t + 1024 * j] = v[8 * s + j];
        __syncthreads();
        // transposed read: butterfly-like stride
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float2 w = CONFLICT ? lds[((t * 8 + j) * (r + 1)) & 8191]
                                    : lds[(t ^ (64 * (r + 1))) + 1024 * ((j + r) & 7)];  // lanes consecutive
          v[8 * s + j] = make_float2(v[8 * s + j].x + w.y, v[8 * s + j].y - w.x);
        }
        __syncthreads();
      }
    }
  }
  float2* o = out + (static_cast<size_t>(blockIdx.y) * L3 + n3) * C;
#pragma unroll
  for (int j = 0; j < 24; ++j) o[t + 1024 * j] = v[j];
}

// A with 512 threads: the 16 gathered inputs stay in registers and each set
// (output residue r) is formed, exchanged and stored in turn; two workgroups
// per CU, so one workgroup's LDS phase overlaps the other's memory phase
template <int ROUNDS, bool STRIDE3 = false>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) passA512(const float* __restrict__ ser, float2* __restrict__ out) {
  __shared__ float2 lds[8192];
  const uint32_t n3 = xcd_col(blockIdx.x, L3);
  const uint32_t t = threadIdx.x;
  float2 v[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const uint32_t np = t + 512 * j;
    const uint32_t n = (np >> 7) * (L2 * L3) + (np & 127) * L3 + n3;
    const uint32_t m = (2 * n + 17 * blockIdx.y) & (NSER - 2);
    v[j] = make_float2(ser[m], ser[m + 1]);
  }
  float2* o = out + (static_cast<size_t>(blockIdx.y) * L3 + n3) * C;
  for (int s = 0; s < 3; ++s) {
    float2 w[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] = make_float2(v[j].x * (s + 1), v[j].y - s);
#pragma unroll
    for (int r = 0; r < ROUNDS; ++r) {
#pragma unroll
      for (int j = 0; j < 16; ++j) lds[t + 512 * j] = w[j];
      __syncthreads();
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const float2 x = lds[(t ^ (64 * (r + 1))) + 512 * ((j + r) & 15)];
        w[j] = make_float2(w[j].x + x.y, w[j].y - x.x);
      }
      __syncthreads();
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      // set-major [r][q], or natural order c = 3 q + r (stride-3 stores, the lines merge in L2)
      const uint32_t q = t + 512 * j;
      o[STRIDE3 ? 3 * q + s : 8192 * s + q] = w[j];
    }
  }
}

// 16 rows c0.. + mirror rows, 256 threads: thread (tile h, n3 quarter)
__global__ void __launch_bounds__(512) passB(const float2* __restrict__ in, float* __restrict__ ps) {
  __shared__ float2 lds[2][L3 * 16];
  const uint32_t blk = blockIdx.x;  // 768 blocks: rows 16 blk .. (c <= C/2)
  const uint32_t c0 = 16 * blk, m0 = C - 16 * blk - 16;
  const float2* src = in + static_cast<size_t>(blockIdx.y) * M;
  const uint32_t t = threadIdx.x;
  // 2 tiles x 256 n3 x 16 rows = 8192 values, 16 per thread: lanes walk rows
  float2 v[16];
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const uint32_t e = t + 512 * u;  // h = e / 4096, n3 = (e / 16) % 256, r = e % 16
    const uint32_t h = e >> 12, n3 = (e >> 4) & 255, r = e & 15;
    v[u] = src[static_cast<size_t>(n3) * C + (h ? m0 : c0) + r];
  }
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const uint32_t e = t + 512 * u;
    lds[e >> 12][((e >> 4) & 255) * 16 + (e & 15)] = v[u];
  }
  __syncthreads();
  // outputs: bins c + C k3 of both tiles, lanes walk rows (16 x 4 B = 64 B pieces)
  float* dst = ps + static_cast<size_t>(blockIdx.y) * M;
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const uint32_t e = t + 512 * u;
    const uint32_t h = e >> 12, k3 = (e >> 4) & 255, r = e & 15;
    const float2 a = lds[h][(k3 * 7 & 255) * 16 + r];
    const uint32_t k = (h ? m0 + r : c0 + r) + C * k3;
    if (k < LIMIT) dst[k] = a.x * a.x + a.y * a.y;
  }
}

// today's pass 1 as a memory shape: 16 consecutive columns n3 x the 64
// non-padding rows n1 of one n2; writes 192 rows x 16 columns
__global__ void __launch_bounds__(256) p1(const float* __restrict__ ser, float2* __restrict__ out) {
  const uint32_t n2 = blockIdx.x / 16, col = n2 * L3 + (blockIdx.x % 16) * 16;
  const uint32_t c = threadIdx.x % 16, tj = threadIdx.x / 16;
  float2 v[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t n = (tj + 16 * q) * (L2 * L3) + col + c;
    const uint32_t m = (2 * n + 17 * blockIdx.y) & (NSER - 2);
    v[q] = make_float2(ser[m], ser[m + 1]);
  }
  float2* o = out + static_cast<size_t>(blockIdx.y) * M + col + c;
#pragma unroll
  for (int q = 0; q < 12; ++q) {
    const float2 a = v[q & 3];
    o[static_cast<size_t>(tj + 16 * q) * (L2 * L3)] = make_float2(a.x + q, a.y);
  }
}

// today's pass 2 as a memory shape: tile (k1, 16 columns n3), 128 rows, in place
__global__ void __launch_bounds__(128) p2(float2* __restrict__ buf) {
  const uint32_t k1 = blockIdx.x / 16, col = k1 * (L2 * L3) + (blockIdx.x % 16) * 16;
  const uint32_t c = threadIdx.x % 16, tj = threadIdx.x / 16;
  float2* b = buf + static_cast<size_t>(blockIdx.y) * M + col + c;
  float2 v[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) v[q] = b[static_cast<size_t>(tj + 8 * q) * L3];
#pragma unroll
  for (int q = 0; q < 16; ++q) b[static_cast<size_t>(tj + 8 * q) * L3] = make_float2(v[15 - q].y, v[q].x);
}

// today's pass 3 as a memory shape: 8 rows + 8 mirror rows of 256, bins c + C k3
__global__ void __launch_bounds__(512) p3(const float2* __restrict__ in, float* __restrict__ ps) {
  const uint32_t c0 = 8 * blockIdx.x, m0 = C - c0 - 8;
  const uint32_t t = threadIdx.x;
  const float2* src = in + static_cast<size_t>(blockIdx.y) * M;
  float* dst = ps + static_cast<size_t>(blockIdx.y) * M;
  float2 v[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const uint32_t e = t + 512 * u;  // h = e / 2048, row r = (e / 256) % 8, n3 = e % 256
    const uint32_t h = e >> 11, r = (e >> 8) & 7, n3 = e & 255;
    v[u] = src[static_cast<size_t>((h ? m0 : c0) + r) * L3 + n3];
  }
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const uint32_t e = t + 512 * u;  // lanes walk rows for the stores: 8 x 4 B pieces
    const uint32_t h = e >> 11, k3 = (e >> 3) & 255, r = e & 7;
    const uint32_t k = (h ? m0 + r : c0 + r) + C * k3;
    if (k < LIMIT) dst[k] = v[u].x * v[u].x + v[u].y;
  }
}

int main() {
  float* ser;
  float2 *buf, *buf2;
  float* ps;
  CHECK(hipMalloc(&ser, sizeof(float) * NSER));
  CHECK(hipMalloc(&buf, sizeof(float2) * M * T));
  CHECK(hipMalloc(&buf2, sizeof(float2) * M * T));
  CHECK(hipMalloc(&ps, sizeof(float) * M * T));
  CHECK(hipMemset(ser, 0, sizeof(float) * NSER));
  CHECK(hipMemset(buf, 0, sizeof(float2) * M * T));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int reps = 40;
  auto timeit = [&](auto launch) -> float {
    launch();
    (void)hipEventRecord(e0);
    for (int r = 0; r < reps; ++r) launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return 1e3f * ms / reps / T;  // per template
  };
  const float tA = timeit([&] { hipLaunchKernelGGL((passA<true>), dim3(L3, T), dim3(1024), 0, 0, ser, buf2); });
  const float tAc3 = timeit([&] { hipLaunchKernelGGL((passA<true, 3, false>), dim3(L3, T), dim3(1024), 0, 0, ser, buf2); });
  const float tAc2 = timeit([&] { hipLaunchKernelGGL((passA<true, 2, false>), dim3(L3, T), dim3(1024), 0, 0, ser, buf2); });
  const float t5123 = timeit([&] { hipLaunchKernelGGL((passA512<3>), dim3(L3, T), dim3(512), 0, 0, ser, buf2); });
  const float t5122 = timeit([&] { hipLaunchKernelGGL((passA512<2>), dim3(L3, T), dim3(512), 0, 0, ser, buf2); });
  const float t512s = timeit([&] { hipLaunchKernelGGL((passA512<3, true>), dim3(L3, T), dim3(512), 0, 0, ser, buf2); });
  const float tA0 = timeit([&] { hipLaunchKernelGGL((passA<false>), dim3(L3, T), dim3(1024), 0, 0, ser, buf2); });
  const float tB = timeit([&] { hipLaunchKernelGGL(passB, dim3(C / 32, T), dim3(512), 0, 0, buf2, ps); });
  const float t1 = timeit([&] { hipLaunchKernelGGL(p1, dim3(L2 * 16, T), dim3(256), 0, 0, ser, buf); });
  const float t2 = timeit([&] { hipLaunchKernelGGL(p2, dim3(L1 * 16, T), dim3(128), 0, 0, buf); });
  const float t3 = timeit([&] { hipLaunchKernelGGL(p3, dim3(C / 16, T), dim3(512), 0, 0, buf, ps); });
  CHECK(hipDeviceSynchronize());
  std::printf("{\"us_per_template\": {\"A_gather_lds_write\": %.2f, \"A_conflict_free_3\": %.2f, \"A_conflict_free_2\": %.2f, \"A512_3\": %.2f, \"A512_2\": %.2f, \"A512_3_stride3\": %.2f, \"A0_gather_write\": %.2f, \"B_tiles_ps\": %.2f, "
              "\"two_pass_total\": %.2f, \"p1\": %.2f, \"p2\": %.2f, \"p3\": %.2f, \"three_pass_total\": %.2f}}\n",
              tA, tAc3, tAc2, t5123, t5122, t512s, tA0, tB, tA + tB, t1, t2, t3, t1 + t2 + t3);
  return 0;
}
