// Memory-cost probe of a fused "pass 2 + pass 3 per k1 slab" FFT (round-4
// review item), not part of the product.
//
// Benchmark plan: M = L1 x L2 x L3 = 192 x 128 x 256 (complex), spectrum bins
// k = k1 + L1 k2 + L1 L2 k3 up to the harmonic limit 5 272 839. A workgroup
// that owns one k1 slab (L2 x L3 = 32 768 values, 256 KB) produces the bins
// k1 + 192 k2 + 24 576 k3: no two of them share a 64-byte line, so a fused
// slab kernel writes its power spectrum as isolated 4-byte stores (or writes
// the slab-ordered spectrum and pays a transpose pass). This probe times,
// on one template's sizes:
//   stream    : read 50 MB + write 21 MB contiguous (the ideal fused kernel)
//   scatter   : read 50 MB contiguous (slab order) + the 21 MB spectrum as
//               the slab's natural-order 4-byte stores
//   p2p3      : the current passes' traffic as streaming copies
//               (read 50 + write 50, read 50 + write 21)
// Build: hipcc --offload-arch=gfx950 -O3 -o build/probe/slab_scatter tools/experiments/slab_scatter.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

#define CHECK(x)                                                                     \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) {                                                           \
      std::printf("HIP error %s at line %d\n", hipGetErrorName(e), __LINE__);        \
      return 1;                                                                      \
    }                                                                                \
  } while (0)

constexpr uint32_t L1 = 192, L2 = 128, L3 = 256, M = L1 * L2 * L3, C = L1 * L2;
constexpr uint32_t LIMIT = 5272839;

// one slab per workgroup: read the slab (contiguous), write its bins
template <bool SCATTER>
__global__ void __launch_bounds__(1024) slab_kernel(const float2* __restrict__ in, float* __restrict__ ps) {
  const uint32_t k1 = blockIdx.x;
  const float2* s = in + static_cast<size_t>(k1) * (L2 * L3);
  float acc = 0.0f;
  for (uint32_t e = threadIdx.x; e < L2 * L3; e += 1024) {
    const float2 v = s[e];
    acc += v.x * v.x + v.y * v.y;
  }
  // outputs: SCATTER -> bin k1 + L1 k2 + C k3 (lanes walk k2: 768 B apart);
  // else a contiguous range of the same size
  for (uint32_t e = threadIdx.x; e < L2 * L3; e += 1024) {
    const uint32_t k2 = e % L2, k3 = e / L2;
    const uint32_t k = SCATTER ? k1 + L1 * k2 + C * k3 : k1 * (L2 * L3) + e;
    if (k < LIMIT) ps[k] = acc + static_cast<float>(e);
  }
}

__global__ void copy_kernel(const float4* __restrict__ in, float4* __restrict__ out, size_t n_in, size_t n_out) {
  const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
  float4 a = make_float4(0, 0, 0, 0);
  for (size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; i < n_in; i += stride) {
    const float4 v = in[i];
    a.x += v.x;
    if (i < n_out) out[i] = make_float4(v.x, v.y, a.x, v.w);
  }
}

int main() {
  float2 *buf, *buf2;
  float* ps;
  CHECK(hipMalloc(&buf, sizeof(float2) * M));
  CHECK(hipMalloc(&buf2, sizeof(float2) * M));
  CHECK(hipMalloc(&ps, sizeof(float) * M));
  CHECK(hipMemset(buf, 0, sizeof(float2) * M));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int reps = 50;
  auto timeit = [&](auto launch) -> float {
    launch();
    (void)hipEventRecord(e0);
    for (int r = 0; r < reps; ++r) launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return 1e3f * ms / reps;
  };
  const size_t n4 = M / 2;  // float4 count of the complex buffer
  const float t_stream = timeit([&] { hipLaunchKernelGGL((slab_kernel<false>), dim3(L1), dim3(1024), 0, 0, buf, ps); });
  const float t_scatter = timeit([&] { hipLaunchKernelGGL((slab_kernel<true>), dim3(L1), dim3(1024), 0, 0, buf, ps); });
  const float t_p2 = timeit([&] {
    hipLaunchKernelGGL(copy_kernel, dim3(4096), dim3(256), 0, 0, reinterpret_cast<const float4*>(buf),
                       reinterpret_cast<float4*>(buf2), n4, n4);
  });
  const float t_p3 = timeit([&] {
    hipLaunchKernelGGL(copy_kernel, dim3(4096), dim3(256), 0, 0, reinterpret_cast<const float4*>(buf2),
                       reinterpret_cast<float4*>(ps), n4, static_cast<size_t>(LIMIT) / 4);
  });
  CHECK(hipDeviceSynchronize());
  std::printf("{\"us\": {\"slab_stream_read50_write21\": %.2f, \"slab_scatter_read50_write21\": %.2f, "
              "\"copy_read50_write50\": %.2f, \"copy_read50_write21\": %.2f, \"p2p3_streaming_floor\": %.2f}}\n",
              t_stream, t_scatter, t_p2, t_p3, t_p2 + t_p3);
  return 0;
}
