// Memory-shape probe of the chirp-z FFT passes (round 5): why does the
// register-staged pass 1 (pass1g_kernel<320>, column stride L2 L3 = 71 680
// complex, 183 MB per transform) move bytes at half the rate of pass 2
// (pass2g_kernel<224>, column stride 320) on the same array?
// Every kernel copies a 183.5 MB complex array out of place with one access
// pattern (no arithmetic); us per copy, single stream, 20 copies timed.
//   cols(R, S): a workgroup of 16 R threads moves R*16 rows x 16 columns,
//               rows tj + R q (q < 16) at row stride S (pass1g / pass2g shape)
//   copy      : float4 streaming copy
// Build: hipcc --offload-arch=gfx950 -O3 stride_probe.hip -o stride_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                        \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      std::printf("HIP error %s at line %d\n", hipGetErrorName(e_), __LINE__);          \
      std::exit(1);                                                                     \
    }                                                                                   \
  } while (0)

constexpr size_t kL1 = 320, kL2 = 224, kL3 = 320;
constexpr size_t kM = kL1 * kL2 * kL3;  // 22 937 600 complex

__global__ void copy4(const float4* __restrict__ in, float4* __restrict__ out, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    out[i] = in[i];
}

// tile = 16 columns x (16 R) rows at stride S; `blocks_per_slab` tiles per
// slab of 16 R rows (pass 2: slabs are the k1 blocks; pass 1: one slab)
template <int R>
__global__ void __launch_bounds__(16 * R) cols(const float2* __restrict__ in, float2* __restrict__ out, uint32_t S,
                                                uint32_t blocks_per_slab, int remap) {
  uint32_t bx = blockIdx.x;
  if (remap) {  // consecutive tiles on one XCD (8 XCDs, round-robin dispatch)
    const uint32_t n = gridDim.x, per = n / 8;
    if (bx < per * 8) bx = (bx % 8) * per + bx / 8;
  }
  const uint32_t slab = bx / blocks_per_slab, cb = bx % blocks_per_slab;
  const int c = threadIdx.x % 16, tj = threadIdx.x / 16;
  const size_t base = (size_t)slab * 16 * R * S + cb * 16 + c + (size_t)tj * S;
  float2 v[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) v[q] = in[base + (size_t)q * R * S];
#pragma unroll
  for (int q = 0; q < 16; ++q) out[base + (size_t)q * R * S] = v[q];
}

// persistent form of cols: grid-stride over the tiles, next tile prefetched
template <int R>
__global__ void __launch_bounds__(16 * R) cols_persist(const float2* __restrict__ in, float2* __restrict__ out,
                                                        uint32_t S, uint32_t blocks_per_slab, uint32_t ntiles) {
  const int c = threadIdx.x % 16, tj = threadIdx.x / 16;
  auto base_of = [&](uint32_t t) {
    const uint32_t slab = t / blocks_per_slab, cb = t % blocks_per_slab;
    return (size_t)slab * 16 * R * S + cb * 16 + c + (size_t)tj * S;
  };
  float2 v[16], w[16];
  uint32_t t = blockIdx.x;
  if (t < ntiles) {
    const size_t b = base_of(t);
#pragma unroll
    for (int q = 0; q < 16; ++q) v[q] = in[b + (size_t)q * R * S];
  }
  while (t < ntiles) {
    const uint32_t nt = t + gridDim.x;
    if (nt < ntiles) {
      const size_t b = base_of(nt);
#pragma unroll
      for (int q = 0; q < 16; ++q) w[q] = in[b + (size_t)q * R * S];
    }
    const size_t b = base_of(t);
#pragma unroll
    for (int q = 0; q < 16; ++q) out[b + (size_t)q * R * S] = v[q];
#pragma unroll
    for (int q = 0; q < 16; ++q) v[q] = w[q];
    t = nt;
  }
}

template <class F>
float time_us(F f) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  f();
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  for (int i = 0; i < 20; ++i) f();
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  CHECK(hipGetLastError());
  return ms * 1000.0f / 20.0f;
}

int main() {
  float2 *in, *out;
  CHECK(hipMalloc(&in, kM * sizeof(float2)));
  CHECK(hipMalloc(&out, kM * sizeof(float2)));
  CHECK(hipMemset(in, 0, kM * sizeof(float2)));
  const double mb = 2.0 * kM * sizeof(float2) / 1e6;
  auto report = [&](const char* name, float us) { std::printf("%-52s %8.1f us  %6.2f TB/s\n", name, us, mb / us); };
  report("copy float4", time_us([&] {
    hipLaunchKernelGGL(copy4, dim3(4096), dim3(256), 0, 0, (const float4*)in, (float4*)out, kM / 2);
  }));
  // pass 1 shape: 320 rows at stride L2 L3 (one slab), 4480 tiles
  const uint32_t S1 = kL2 * kL3;
  report("pass1 shape  R=20 rows 320 stride 71680", time_us([&] {
    hipLaunchKernelGGL(cols<20>, dim3(S1 / 16), dim3(320), 0, 0, in, out, S1, S1 / 16, 0);
  }));
  report("pass1 shape, XCD-remapped tiles", time_us([&] {
    hipLaunchKernelGGL(cols<20>, dim3(S1 / 16), dim3(320), 0, 0, in, out, S1, S1 / 16, 1);
  }));
  report("pass1 shape, persistent 1024 wgs + prefetch", time_us([&] {
    hipLaunchKernelGGL(cols_persist<20>, dim3(1024), dim3(320), 0, 0, in, out, S1, S1 / 16, S1 / 16);
  }));
  // pass 2 shape: slabs of 224 rows at stride 320 (L1 slabs x L3/16 tiles)
  report("pass2 shape  R=14 rows 224 stride 320", time_us([&] {
    hipLaunchKernelGGL(cols<14>, dim3(kL1 * kL3 / 16), dim3(224), 0, 0, in, out, (uint32_t)kL3, (uint32_t)(kL3 / 16), 0);
  }));
  // pass 1 shape with fewer rows per tile but the same span: 64 rows at stride 5 L2 L3 (R=4)
  report("64 rows at stride 358400 (same span, 5x tiles)", time_us([&] {
    hipLaunchKernelGGL(cols<4>, dim3(5 * S1 / 16), dim3(64), 0, 0, in, out, 5 * S1, 5 * S1 / 16, 0);
  }));
  // 320 rows at a small stride (tile span 320 x 2.5 KB), as many tiles
  report("320 rows at stride 320 (pass2-like span)", time_us([&] {
    hipLaunchKernelGGL(cols<20>, dim3(kL1 * kL2 * kL3 / 320 / 16), dim3(320), 0, 0, in, out, (uint32_t)kL3,
                       (uint32_t)(kL3 / 16), 0);
  }));
  // bench geometry pass 1 (192 rows, stride 32768) on a 50 MB array, for reference
  CHECK(hipFree(in));
  CHECK(hipFree(out));
  return 0;
}
