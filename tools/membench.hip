// Memory-pattern microbenchmark for the FFT pass design (not part of the product).
// Measures achievable bandwidth on gfx950 for:
//   copy      : float4 streaming copy
//   colblk W  : "column block" access of the FFT column passes: a workgroup reads
//               L rows x W complex (8 B) with row stride S complex, writes them back
//               in place (pass-2 pattern), with an LDS round trip
// Usage: membench  (prints one line per pattern)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../csrc/hip/fft_block.hpp"
using namespace brp::hipk;

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorName(e), __LINE__); return 1; } } while (0)

__global__ void copy_kernel(const float4* __restrict__ in, float4* __restrict__ out, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) out[i] = in[i];
}

// WG handles a block of W consecutive columns x L rows (row stride S), in place.
template <int L, int W, int NT>
__global__ void __launch_bounds__(NT) colblk_kernel(float2* buf, int S, int nblk_per_row) {
  __shared__ float2 lds[L * W];
  const int row_blk = blockIdx.x / nblk_per_row;  // which slab
  const int cb = blockIdx.x % nblk_per_row;
  float2* base = buf + (size_t)row_blk * L * S + cb * W;
  for (int e = threadIdx.x; e < L * W; e += NT) {
    const int r = e / W, c = e % W;
    lds[e] = base[(size_t)r * S + c];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < L * W; e += NT) {
    const int r = e / W, c = e % W;
    float2 v = lds[(e + W) % (L * W)];
    v.x += 1.0f;
    base[(size_t)r * S + c] = v;
  }
}

// same but float4 accesses (2 complex per lane)
template <int L, int W, int NT>
__global__ void __launch_bounds__(NT) colblk4_kernel(float4* buf, int S2, int nblk_per_row) {
  __shared__ float4 lds[L * W / 2];
  const int row_blk = blockIdx.x / nblk_per_row;
  const int cb = blockIdx.x % nblk_per_row;
  float4* base = buf + (size_t)row_blk * L * S2 + cb * (W / 2);
  constexpr int W2 = W / 2;
  for (int e = threadIdx.x; e < L * W2; e += NT) {
    const int r = e / W2, c = e % W2;
    lds[e] = base[(size_t)r * S2 + c];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < L * W2; e += NT) {
    const int r = e / W2, c = e % W2;
    float4 v = lds[(e + W2) % (L * W2)];
    v.x += 1.0f;
    base[(size_t)r * S2 + c] = v;
  }
}

// pass-2 shaped kernel with the real block FFT in the middle (ABL: 0 full, 1 no FFT)
template <int L, int ABL>
__global__ void __launch_bounds__(16 * (L / 16)) colfft_kernel(float2* buf, int S, int nblk_per_row, const float2* st) {
  constexpr int TPC = L / 16;
  using Lay = BlockLayout<L, 16, TPC, false>;
  __shared__ float2 smem[Lay::kLds + kTwPad<L>];
  float2* data = smem;
  float2* twl = smem + Lay::kLds;
  const int row_blk = blockIdx.x / nblk_per_row;
  const int cb = blockIdx.x % nblk_per_row;
  float2* base = buf + (size_t)row_blk * L * S + cb * 16;
  int c, tj;
  Lay::coords(threadIdx.x, c, tj);
  for (int r = tj; r < L; r += TPC) data[Lay::idx(r, c)] = base[(size_t)r * S + c];
  copy_stage_twiddles<L>(twl, st);
  __syncthreads();
  if (ABL == 0) BlockFFT<L, 16, TPC, false>::run(data, twl);
  for (int r = tj; r < L; r += TPC) base[(size_t)r * S + c] = data[Lay::idx(r, c)];
}

template <typename F>
float time_it(F f, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  f();
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(a);
  for (int i = 0; i < reps; ++i) f();
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

__global__ void copy2_kernel(const float2* __restrict__ in, float2* __restrict__ out, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) out[i] = in[i];
}

int main(int argc, char** argv) {
  const size_t M = 6291456;  // complex elements of one template (50 MB)
  const int B = argc > 1 ? atoi(argv[1]) : 4;  // templates (16: 800 MB, beyond the 256 MB Infinity Cache)
  printf("buffer %d templates = %.0f MB\n", B, B * M * 8 / 1e6);
  const size_t n = M * B;
  float2 *buf, *buf2;
  CHECK(hipMalloc(&buf, n * sizeof(float2)));
  CHECK(hipMalloc(&buf2, n * sizeof(float2)));
  CHECK(hipMemset(buf, 0, n * sizeof(float2)));
  const double bytes_rw = 2.0 * n * sizeof(float2);
  {
    const size_t n4 = n / 2;
    float ms = time_it([&] { hipLaunchKernelGGL(copy_kernel, dim3(4096), dim3(256), 0, 0, (const float4*)buf, (float4*)buf2, n4); }, 20);
    printf("copy float4           %8.3f ms  %6.2f TB/s\n", ms, bytes_rw / ms / 1e9);
    ms = time_it([&] { hipLaunchKernelGGL(copy2_kernel, dim3(4096), dim3(256), 0, 0, (const float2*)buf, buf2, n); }, 20);
    printf("copy float2           %8.3f ms  %6.2f TB/s\n", ms, bytes_rw / ms / 1e9);
  }
  // pass-2 like: L=128 rows, stride S=256 complex (2 KB), slabs = M/(128*256)
  {
    constexpr int L = 128, W = 16, NT = 128;
    const int S = 256;
    const int slabs = n / (L * S);
    const int nbr = S / W;
    float ms = time_it([&] { hipLaunchKernelGGL((colblk_kernel<L, W, NT>), dim3(slabs * nbr), dim3(NT), 0, 0, buf, S, nbr); }, 20);
    printf("colblk L128 W16 NT128 %8.3f ms  %6.2f TB/s\n", ms, bytes_rw / ms / 1e9);
  }
  {
    constexpr int L = 128, W = 16, NT = 256;
    const int S = 256;
    const int slabs = n / (L * S);
    const int nbr = S / W;
    float ms = time_it([&] { hipLaunchKernelGGL((colblk_kernel<L, W, NT>), dim3(slabs * nbr), dim3(NT), 0, 0, buf, S, nbr); }, 20);
    printf("colblk L128 W16 NT256 %8.3f ms  %6.2f TB/s\n", ms, bytes_rw / ms / 1e9);
  }
  {
    constexpr int L = 128, W = 32, NT = 256;
    const int S = 256;
    const int slabs = n / (L * S);
    const int nbr = S / W;
    float ms = time_it([&] { hipLaunchKernelGGL((colblk_kernel<L, W, NT>), dim3(slabs * nbr), dim3(NT), 0, 0, buf, S, nbr); }, 20);
    printf("colblk L128 W32 NT256 %8.3f ms  %6.2f TB/s\n", ms, bytes_rw / ms / 1e9);
  }
  {
    constexpr int L = 128, W = 16, NT = 128;
    const int S2 = 128;
    const int slabs = n / (L * 256);
    const int nbr = 256 / W;
    float ms = time_it([&] { hipLaunchKernelGGL((colblk4_kernel<L, W, NT>), dim3(slabs * nbr), dim3(NT), 0, 0, (float4*)buf, S2, nbr); }, 20);
    printf("colblk4 L128 W16 NT128%8.3f ms  %6.2f TB/s\n", ms, bytes_rw / ms / 1e9);
  }
  {
    constexpr int L = 128, W = 64, NT = 256;
    const int S = 256;
    const int slabs = n / (L * S);
    const int nbr = S / W;
    float ms = time_it([&] { hipLaunchKernelGGL((colblk_kernel<L, W, NT>), dim3(slabs * nbr), dim3(NT), 0, 0, buf, S, nbr); }, 20);
    printf("colblk L128 W64 NT256 %8.3f ms  %6.2f TB/s\n", ms, bytes_rw / ms / 1e9);
  }
  // contiguous rows (pass-3 like): W=1 column block of 256-long rows == contiguous 2KB rows
  {
    constexpr int L = 16, W = 256, NT = 256;  // 16 rows x 256 contiguous
    const int S = 256;
    const int slabs = n / (L * S);
    float ms = time_it([&] { hipLaunchKernelGGL((colblk_kernel<L, W, NT>), dim3(slabs), dim3(NT), 0, 0, buf, S, 1); }, 20);
    printf("rows 16x256 NT256     %8.3f ms  %6.2f TB/s\n", ms, bytes_rw / ms / 1e9);
  }
  {
    float2* st;
    CHECK(hipMalloc(&st, 4096 * sizeof(float2)));
    CHECK(hipMemset(st, 0, 4096 * sizeof(float2)));
    const int S = 256;
    const int nbr = S / 16;
    {
      const int slabs = n / (128 * S);
      float ms = time_it([&] { hipLaunchKernelGGL((colfft_kernel<128, 1>), dim3(slabs * nbr), dim3(128), 0, 0, buf, S, nbr, st); }, 20);
      printf("colfft L128 noFFT     %8.3f ms  %6.2f TB/s\n", ms, bytes_rw / ms / 1e9);
      ms = time_it([&] { hipLaunchKernelGGL((colfft_kernel<128, 0>), dim3(slabs * nbr), dim3(128), 0, 0, buf, S, nbr, st); }, 20);
      printf("colfft L128 FFT       %8.3f ms  %6.2f TB/s\n", ms, bytes_rw / ms / 1e9);
    }
    {
      const int slabs = n / (192 * S);
      float ms = time_it([&] { hipLaunchKernelGGL((colfft_kernel<192, 1>), dim3(slabs * nbr), dim3(192), 0, 0, buf, S, nbr, st); }, 20);
      printf("colfft L192 noFFT     %8.3f ms  %6.2f TB/s\n", ms, bytes_rw / ms / 1e9);
      ms = time_it([&] { hipLaunchKernelGGL((colfft_kernel<192, 0>), dim3(slabs * nbr), dim3(192), 0, 0, buf, S, nbr, st); }, 20);
      printf("colfft L192 FFT       %8.3f ms  %6.2f TB/s\n", ms, bytes_rw / ms / 1e9);
    }
    {
      const int slabs = n / (256 * S);
      float ms = time_it([&] { hipLaunchKernelGGL((colfft_kernel<256, 1>), dim3(slabs * nbr), dim3(256), 0, 0, buf, S, nbr, st); }, 20);
      printf("colfft L256 noFFT     %8.3f ms  %6.2f TB/s\n", ms, bytes_rw / ms / 1e9);
      ms = time_it([&] { hipLaunchKernelGGL((colfft_kernel<256, 0>), dim3(slabs * nbr), dim3(256), 0, 0, buf, S, nbr, st); }, 20);
      printf("colfft L256 FFT       %8.3f ms  %6.2f TB/s\n", ms, bytes_rw / ms / 1e9);
    }
  }
  (void)hipFree(buf);
  (void)hipFree(buf2);
  return 0;
}
