// Experiment: can matrix cores replace an LDS exchange in
// the pass-3 row FFT? The 256-point row FFT as two complex 16x16x16 products
// with v_mfma_f32_16x16x4_f32, X_k (k = 16 k1 + k2) = sum_n1 W16^{n1 k1}
// W256^{n1 k2} sum_n2 x[n1 + 16 n2] W16^{n2 k2}, against the product's LDS
// Stockham radix-16 x 16 row FFT (fft_block.hpp), same loads and |X|^2 stores.
//
// MFMA operand maps (cdna_hip_programming.md §3, f32 16x16x4): lane l holds
// A[l & 15][k = l >> 4] and B[k = l >> 4][l & 15] of each K-step; C/D holds
// row 4 (l >> 4) + r, column l & 15 in register r. The first product
// Y = X F takes A = x[l + 64 s] (coalesced row loads) and B = F. The second,
// Z = F (T o Y), sums over Y's row index; with the K order of step s permuted
// to rows {4 g + s}, lane group g's operand is its own accumulator register s,
// so no data moves between the products (no LDS at all in the MFMA kernel).
//
// Build + run (GPU box): hipcc --offload-arch=gfx950 -O3 -std=c++17 -I csrc \
//   tools/experiments/mfma_dft16/mfma_rowfft.hip -o /tmp/mfma_rowfft && /tmp/mfma_rowfft
#include <hip/hip_runtime.h>

#include <cmath>
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "hip/fft_block.hpp"

using namespace brp::hipk;

#define CHECK(x)                                                                 \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                              \
    }                                                                            \
  } while (0)

constexpr int L = 256;
constexpr int ROWS = 16;  // rows per workgroup of the LDS kernel (pass 3: 2 x 8)
constexpr int TPC = 16;

// ---- (A) LDS Stockham: the product's row FFT core
__global__ void __launch_bounds__(ROWS * TPC) lds_rowfft(const float2* __restrict__ in, float* __restrict__ out,
                                                         const float2* __restrict__ st, int nrows) {
  using Lay = BlockLayout<L, ROWS, TPC, true>;
  __shared__ __attribute__((aligned(16))) float2 smem[Lay::kLds + kTwPad<L> + kTwRowExtra<L>];
  float2* data = smem;
  float2* twl = smem + Lay::kLds;
  const int row0 = blockIdx.x * ROWS;
  int slot, tj;
  Lay::coords(threadIdx.x, slot, tj);
  const float4* src = reinterpret_cast<const float4*>(in + static_cast<size_t>(row0 + slot) * L);
  for (int r = tj; r < L / 2; r += TPC) {
    const float4 v = src[r];
    data[Lay::idx(2 * r, slot)] = make_float2(v.x, v.y);
    data[Lay::idx(2 * r + 1, slot)] = make_float2(v.z, v.w);
  }
  copy_row_twiddles<L>(twl, st);
  __syncthreads();
  BlockFFT<L, ROWS, TPC, true>::run(data, twl);
  float* o = out + static_cast<size_t>(row0 + slot) * L;
  for (int k = tj; k < L; k += TPC) {
    const float2 z = data[Lay::idx(k, slot)];
    o[k] = z.x * z.x + z.y * z.y;
  }
}

// ---- (B) MFMA: one wave per row, grid-stride over rows, two rows in flight
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) mfma_rowfft(const float2* __restrict__ in, float* __restrict__ out,
                                                   const float2* __restrict__ tabs, int nrows) {
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, c = lane & 15;
  // constants (exact host values): first-product B = F[g + 4 s][c], second-product
  // A = F[c][4 g + s], twiddles T[4 g + r][c]
  float f1r[4], f1i[4], f1n[4], f2r[4], f2i[4], f2n[4], tr[4], ti[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const float2 a = tabs[((g + 4 * s) * c) % 16];
    f1r[s] = a.x; f1i[s] = a.y; f1n[s] = -a.y;
    const float2 b = tabs[(c * (4 * g + s)) % 16];
    f2r[s] = b.x; f2i[s] = b.y; f2n[s] = -b.y;
    const float2 t = tabs[16 + (4 * g + s) * c];  // W256^{n1 k2}
    tr[s] = t.x; ti[s] = t.y;
  }
  const int waves = gridDim.x * (blockDim.x / 64);
  for (int row = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); row < nrows; row += waves) {
    const float2* x = in + static_cast<size_t>(row) * L;
    float2 xv[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) xv[s] = x[lane + 64 * s];
    f32x4 yr = {0, 0, 0, 0}, yi = {0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      yr = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[s].x, f1r[s], yr, 0, 0, 0);
      yi = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[s].x, f1i[s], yi, 0, 0, 0);
      yr = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[s].y, f1n[s], yr, 0, 0, 0);
      yi = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[s].y, f1r[s], yi, 0, 0, 0);
    }
    // twiddle T o Y (lane holds Y[4 g + r][c])
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float a = yr[r], b = yi[r];
      yr[r] = a * tr[r] - b * ti[r];
      yi[r] = a * ti[r] + b * tr[r];
    }
    f32x4 zr = {0, 0, 0, 0}, zi = {0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < 4; ++s) {  // K = {4 g + s}: B operand = own register s
      zr = __builtin_amdgcn_mfma_f32_16x16x4f32(f2r[s], yr[s], zr, 0, 0, 0);
      zi = __builtin_amdgcn_mfma_f32_16x16x4f32(f2r[s], yi[s], zi, 0, 0, 0);
      zr = __builtin_amdgcn_mfma_f32_16x16x4f32(f2n[s], yi[s], zr, 0, 0, 0);
      zi = __builtin_amdgcn_mfma_f32_16x16x4f32(f2i[s], yr[s], zi, 0, 0, 0);
    }
    // Z[k1 = 4 g + r][k2 = c] -> k = 16 k1 + k2
    float* o = out + static_cast<size_t>(row) * L;
#pragma unroll
    for (int r = 0; r < 4; ++r) o[64 * g + 16 * r + c] = zr[r] * zr[r] + zi[r] * zi[r];
  }
}

int main() {
  const int nrows = 2 * 24576;  // one benchmark template's pass-3 rows (C = 24576, pairs)
  const int reps = 200;
  std::vector<float2> h_in(static_cast<size_t>(nrows) * L);
  unsigned s = 12345;
  for (auto& v : h_in) {
    s = s * 1664525u + 1013904223u;
    const float a = (s >> 8) * (1.0f / 16777216.0f) - 0.5f;
    s = s * 1664525u + 1013904223u;
    const float b = (s >> 8) * (1.0f / 16777216.0f) - 0.5f;
    v = make_float2(a, b);
  }
  const double pi = 3.14159265358979323846;
  auto root = [&](long j, long n) {
    const double a = -2.0 * pi * static_cast<double>(j % n) / static_cast<double>(n);
    return make_float2(static_cast<float>(std::cos(a)), static_cast<float>(std::sin(a)));
  };
  // stage table for the LDS kernel (padded + q-major block, as stage_table_rows)
  std::vector<float2> st(L + L / 16 + 1, make_float2(0, 0));
  for (int e = 0; e < L; ++e) st[e + (e >> 4)] = root(e, L);
  for (int q = 1; q < 16; ++q)
    for (int jm = 0; jm < L / 16; ++jm) st.push_back(root(static_cast<long>(jm) * q, L));
  // MFMA tables: W16^j (16) then W256^j (256)
  std::vector<float2> tabs(16 + 256);
  for (int j = 0; j < 16; ++j) tabs[j] = root(j, 16);
  for (int j = 0; j < 256; ++j) tabs[16 + j] = root(j, 256);

  float2 *d_in, *d_st, *d_tabs;
  float *d_a, *d_b;
  CHECK(hipMalloc(&d_in, h_in.size() * sizeof(float2)));
  CHECK(hipMalloc(&d_a, static_cast<size_t>(nrows) * L * sizeof(float)));
  CHECK(hipMalloc(&d_b, static_cast<size_t>(nrows) * L * sizeof(float)));
  CHECK(hipMalloc(&d_st, st.size() * sizeof(float2)));
  CHECK(hipMalloc(&d_tabs, tabs.size() * sizeof(float2)));
  CHECK(hipMemcpy(d_in, h_in.data(), h_in.size() * sizeof(float2), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_st, st.data(), st.size() * sizeof(float2), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_tabs, tabs.data(), tabs.size() * sizeof(float2), hipMemcpyHostToDevice));

  auto run_a = [&] { hipLaunchKernelGGL(lds_rowfft, dim3(nrows / ROWS), dim3(ROWS * TPC), 0, 0, d_in, d_a, d_st, nrows); };
  const int mfma_blocks = 256 * 8;  // 8 workgroups of 4 waves per CU, grid-stride
  auto run_b = [&] { hipLaunchKernelGGL(mfma_rowfft, dim3(mfma_blocks), dim3(256), 0, 0, d_in, d_b, d_tabs, nrows); };
  run_a();
  run_b();
  CHECK(hipDeviceSynchronize());
  std::vector<float> ha(static_cast<size_t>(nrows) * L), hb(ha.size());
  CHECK(hipMemcpy(ha.data(), d_a, ha.size() * sizeof(float), hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(hb.data(), d_b, hb.size() * sizeof(float), hipMemcpyDeviceToHost));
  // host double DFT of a few rows
  double err_a = 0, err_b = 0, scale = 0;
  for (int row : {0, 1, 777, nrows - 1}) {
    for (int k = 0; k < L; ++k) {
      std::complex<double> acc = 0;
      for (int n = 0; n < L; ++n) {
        const float2 v = h_in[static_cast<size_t>(row) * L + n];
        acc += std::complex<double>(v.x, v.y) * std::polar(1.0, -2.0 * pi * ((static_cast<long>(n) * k) % L) / L);
      }
      const double p = std::norm(acc);
      scale = std::max(scale, p);
      err_a = std::max(err_a, std::fabs(ha[static_cast<size_t>(row) * L + k] - p));
      err_b = std::max(err_b, std::fabs(hb[static_cast<size_t>(row) * L + k] - p));
    }
  }
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  double ms_a = 0, ms_b = 0;
  for (int round = 0; round < 3; ++round) {
    float t;
    CHECK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) run_a();
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&t, e0, e1));
    ms_a = round ? std::min(ms_a, static_cast<double>(t)) : t;
    CHECK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) run_b();
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&t, e0, e1));
    ms_b = round ? std::min(ms_b, static_cast<double>(t)) : t;
  }
  std::printf("{\"rows\": %d, \"lds_us\": %.2f, \"mfma_us\": %.2f, \"lds_max_abs_err_rel\": %.3g, "
              "\"mfma_max_abs_err_rel\": %.3g}\n",
              nrows, 1e3 * ms_a / reps, 1e3 * ms_b / reps, err_a / scale, err_b / scale);
  return 0;
}
