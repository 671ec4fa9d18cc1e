// Two-pass packed real FFT for the benchmark geometry (M = C x L3 complex with
// C = L1 L2 = 3 * 8192 = 24576, L3 = 256, padding >= 3x).
//
// The three-pass plan (fft_passes.hip) moves the 50 MB complex array through
// memory four times per template: pass 1 writes it, pass 2 reads and writes it,
// pass 3 reads it. Here passes 1 and 2 are one column transform of C points per
// column n3, held by one workgroup, written transposed ([n3][c], contiguous), and
// pass B (pass3_kernel with TP) reads pass 3's rows as [n3][rows] tiles: 100 MB
// less traffic per template (memory-shape probe: tools/experiments/two_pass_probe.hip).
//
// Column transform (index algebra): Z[c + C k3] = sum_n3 W_L3^{n3 k3} W_M^{n3 c} X_n3[c],
//   X_n3[c] = sum_{n' < 8192} x[256 n' + n3] W_C^{n' c}
// (inputs n' >= C/3 lie in the zero padding). With c = 3 q + r (set r < 3):
//   X_n3[3 q + r] = sum_{n'} (x[n'] W_C^{n' r}) W_8192^{n' q},
// three 8192-point transforms of the twiddled column. Each is split as
// n' = 8 t + j (t < 1024, j < 8), q = k1 + 1024 k2:
//   Y[k1 + 1024 k2] = sum_j W_8^{j k2} W_8192^{j k1} sum_t y[8 t + j] W_1024^{t k1}
// i.e. 8 LDS-resident FFT-1024 columns (Stockham radix 16, 8, 8; the first
// stage straight from the gathered registers), then per row k1 a radix-8 DFT
// over the 8 columns. The gathered column stays in registers across the three
// sets (32 VGPRs; the kernel fits 128 VGPRs without spills at two workgroups
// per CU).
//
// Output layout (pass B reads it): within column n3, row c = 3 q + r is stored
// at tp_pos(c) = 24 (q / 8) + 8 r + q % 8 (kTpBlock = 24), so a set's 8
// consecutive q are one 64-B piece and rows [24 b, 24 b + 24) one 192-B block.
// Replaces the reference's cuFFT call and resampling kernels
// (cuda/app/demod_binary_cuda.cu:849-965, cuda/app/demod_binary_cuda.cuh:69-184).
#include <string>
#include <vector>

#include "fft_block.hpp"
#include "fft_kernels.hpp"
#include "two_pass_check.hpp"

namespace brp {
namespace hipk {

namespace {

constexpr int kAT = 512;                // threads per column workgroup
constexpr int kACols = 8;               // FFT-1024 columns (j)
constexpr int kALen = 1024;             // FFT length per column (t)
constexpr uint32_t kAC = 24576;         // C
constexpr uint32_t kAL3 = 256;          // L3 (columns n3)
constexpr uint32_t kAL2L3 = 128 * 256;  // input stride of n1
// neighbouring columns per workgroup (build switch): 2 halves the series lines
// the column gathers fetch per column (a line holds 16 columns), at one
// workgroup per CU instead of two
#ifndef BRP_PA_COLS
#define BRP_PA_COLS 1
#endif
constexpr int kNC = BRP_PA_COLS;
static_assert(kNC == 1 || kNC == 2, "columns per pass-A workgroup");

// Speed-of-light ablations for experiment builds (scripts/build_variant.sh,
// wrong results): BRP_ABLATE_PA_RES drops the resampling arithmetic,
// BRP_ABLATE_PA_FFT the LDS stages and DFTs, BRP_ABLATE_PA_GATHER the series loads.
#ifdef BRP_ABLATE_PA_RES
constexpr bool kAblRes = true;
#else
constexpr bool kAblRes = false;
#endif
#ifdef BRP_ABLATE_PA_FFT
constexpr bool kAblFft = true;
#else
constexpr bool kAblFft = false;
#endif
#ifdef BRP_ABLATE_PA_GATHER
constexpr bool kAblGather = true;
#else
constexpr bool kAblGather = false;
#endif

// column-interleaved, XOR-swizzled 1024 x 8 block: the 8 lanes of a row touch
// a permutation of its 64 B (stage reads / writes conflict-free); the final
// read (lanes walk rows, one column) spreads over all 64 banks
__host__ __device__ inline int a_idx(int t, int j) { return t * kACols + (j ^ ((t >> 2) & 7)); }

// pass A's output position of (set r, row k1, output k2) within a column:
// q = k1 + 1024 k2, c = 3 q + r, tp_pos(c)
__host__ __device__ inline uint32_t pa_store_pos(uint32_t r, uint32_t k1, uint32_t k2) {
  constexpr uint32_t kQb = kTpBlock / 3;  // q per layout block
  return kTpBlock * (k1 / kQb) + kQb * r + (k1 % kQb) + 3072u * k2;  // q + 1024: 1024 / kQb blocks
}
// Stockham row written by stage (radix R, span Ns) for butterfly jp, output p
__host__ __device__ inline int a_stage_row(int Ns, int R, int jp, int p) { return (jp / Ns) * Ns * R + (jp % Ns) + Ns * p; }

// radix-8 Stockham stage (Ns = 16, 128) of the 8 FFT-1024 columns, LDS -> LDS:
// butterflies j' = tj, tj + 64 of column c
template <int Ns>
__device__ __forceinline__ void a_stage(float2* data, const float2* __restrict__ w1024, int c, int tj) {
  float2 v[2][8];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int jp = tj + 64 * h;
#pragma unroll
    for (int p = 0; p < 8; ++p) v[h][p] = data[a_idx(jp + 128 * p, c)];
    const int jm = jp % Ns;
#pragma unroll
    for (int p = 1; p < 8; ++p) v[h][p] = cmul(v[h][p], w1024[(jm * p * (kALen / (8 * Ns))) & (kALen - 1)]);
    if constexpr (!kAblFft) Dft<8>::run(v[h]);
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int jp = tj + 64 * h;
#pragma unroll
    for (int p = 0; p < 8; ++p) data[a_idx(a_stage_row(Ns, 8, jp, p), c)] = v[h][p];
  }
  __syncthreads();
}

// LDS: exactly the 64 KB column block (the twiddle tables and the sine LUT are
// read through the caches; the block-sum scratch reuses the block at the end)
__global__ void __launch_bounds__(kAT) __attribute__((amdgpu_waves_per_eu(kNC == 1 ? 4 : 2, 8))) pass_a_kernel(PassAArgs a) {
  __shared__ __attribute__((aligned(16))) float2 data[kALen * kACols];
  const float2* __restrict__ w1024 = a.w1024;  // W_1024^e
  const float2* __restrict__ w48 = a.w48;      // W_48^e  (= W_C^{512 e})
  const float* __restrict__ lut_s = a.lut_sin;
  const float* __restrict__ lut_c = a.lut_cos;

  const int b = blockIdx.y;
  const uint32_t n3b = kNC * xcd_remap(blockIdx.x, gridDim.x);  // neighbouring columns share series lines: one XCD
  const int tid = static_cast<int>(threadIdx.x);
  if (a.reset != nullptr && blockIdx.x == 0 && blockIdx.y == 0 && tid == 0) *a.reset = 0;

  const TemplateDev td = a.tmpl[b];
  // gather rows t = tj + 64 u (u < 16) of column j = c: n' = 8 t + c ->
  // n1 = n' / 128, n2 = n' % 128 (complex sample 256 n' + n3)
  const int c0 = tid % kACols;
  const int tj0 = tid / kACols;
  const bool fast = a.n_unpadded <= (1u << 23);
  const float* series = a.series + static_cast<size_t>(td.wu) * a.n_unpadded;
  const int last = static_cast<int>(a.n_unpadded) - 1;
  float fsum = 0.0f;
  float2 x[kNC][16];
  // two halves of 8 rows (16 indices and loads in flight each, per column)
#pragma unroll
  for (int hf = 0; hf < 2; ++hf) {
    int idx[kNC][16];
#pragma unroll
    for (int v = 0; v < 8; ++v) {
      const int u = 8 * hf + v;
      const uint32_t np = 8u * (tj0 + 64u * u) + c0;
#pragma unroll
      for (int h = 0; h < 2 * kNC; ++h) {  // samples m0 .. m0 + 2 kNC - 1: the columns' pairs, adjacent
        const uint32_t m = 2u * ((np >> 7) * kAL2L3 + (np & 127u) * kAL3 + n3b) + h;
        int i = -1;
        if (m < td.n_steps) {
          if constexpr (kAblRes) {
            i = min(static_cast<int>(m), last);
          } else {
            const float dt = resamp_del_t(m, td.p, lut_s, lut_c);
            i = min(max(fast ? resamp_nearest_f(m, dt) : resamp_nearest(m, dt), 0), last);
          }
        }
        idx[h >> 1][2 * v + (h & 1)] = i;
      }
    }
#pragma unroll
    for (int cc = 0; cc < kNC; ++cc) {
      float raw[16];
#pragma unroll
      for (int e = 0; e < 16; ++e)
        raw[e] = kAblGather ? static_cast<float>(idx[cc][e]) : series[idx[cc][e] < 0 ? 0 : idx[cc][e]];
#pragma unroll
      for (int v = 0; v < 8; ++v) {
        const float x0 = idx[cc][2 * v] < 0 ? 0.0f : raw[2 * v] - td.mu0;
        const float x1 = idx[cc][2 * v + 1] < 0 ? 0.0f : raw[2 * v + 1] - td.mu0;
        fsum += x0 + x1;
        x[cc][8 * hf + v] = make_float2(x0, x1);
      }
    }
  }

  // output origin, uniform: kept in SGPRs (stores are SGPR base + lane offset)
  // (readfirstlane returns a signed int: each half goes back through uint32_t
  // before widening, or a low half >= 2^31 would sign-extend over the high half
  // -- the out-of-range stores the first forms of this kernel made whenever the
  // column's address had bit 31 set, profiles/two_pass_r4.txt)
#pragma unroll 1
  for (int cc = 0; cc < kNC; ++cc) {
  const uint32_t n3 = n3b + cc;
  char* outb;
  {
    const uint64_t o = reinterpret_cast<uint64_t>(a.out + (static_cast<size_t>(b) * kAL3 + n3) * kAC);
    const uint32_t lo = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(static_cast<uint32_t>(o))));
    const uint32_t hi = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(static_cast<uint32_t>(o >> 32))));
    outb = reinterpret_cast<char*>((static_cast<uint64_t>(hi) << 32) | lo);
  }
#pragma unroll 1
  for (int r = 0; r < 3; ++r) {
    // thread coordinates made opaque per set: otherwise the set's LDS
    // addresses are hoisted out of the loop and held in registers
    int tr = tid;
    asm volatile("" : "+v"(tr));
    const int c = tr % kACols, tj = tr / kACols;
    // set twiddle y = x W_C^{(8 t + j) r} = x * W_C^{(8 tj + c) r} * W_48^{u r}
    // (W_C^e = W_4M^{1024 e}); stage 1 (radix 16, Ns = 1) in registers:
    // butterfly j' = tj reads rows t = tj + 64 u, exactly the gathered ones
    const float2 ar = tw_lookup32(a.tw, 1024u * r * (8u * tj + c));
    float2 v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = (r == 0) ? x[cc][u] : cmul(x[cc][u], u == 0 ? ar : cmul(ar, w48[(u * r) % 48]));
    if constexpr (!kAblFft) Dft<16>::run(v);
    if (r != 0 || cc != 0) __syncthreads();  // the previous set's final reads are done
#pragma unroll
    for (int p = 0; p < 16; ++p) data[a_idx(a_stage_row(1, 16, tj, p), c)] = v[p];
    __syncthreads();
    if constexpr (!kAblFft) {
      a_stage<16>(data, w1024, c, tj);
      a_stage<128>(data, w1024, c, tj);
    }
    // final: rows k1 = tid, tid + 512 of the 8 columns, twiddle W_8192^{j k1},
    // radix 8 over j -> k2; q = k1 + 1024 k2, c = 3 q + r
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const int k1 = tr + kAT * hh;
      float2 z[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) z[j] = data[a_idx(k1, j)];
      float2 wp[3];  // W_8192^{k1 2^i} (W_4M^{3072 e}), exact table products
#pragma unroll
      for (int i = 0; i < 3; ++i) wp[i] = tw_lookup32(a.tw, (3072u << i) * static_cast<uint32_t>(k1));
#pragma unroll
      for (int j = 1; j < 8; ++j) {
        float2 w = make_float2(1.f, 0.f);
        bool first = true;
#pragma unroll
        for (int i = 0; i < 3; ++i)
          if (j & (1 << i)) {
            w = first ? wp[i] : cmul(w, wp[i]);
            first = false;
          }
        z[j] = cmul(z[j], w);
      }
      if constexpr (!kAblFft) Dft<8>::run(z);
      // output twiddle W_M^{n3 c} = W_M^{n3 (3 k1 + r)} W_M^{3072 n3 k2}
      const float2 wo = tw_lookup32(a.tw, 4u * n3 * (3u * k1 + r));
      uint32_t off = pa_store_pos(r, k1, 0) * sizeof(float2);
#pragma unroll
      for (int k2 = 0; k2 < 8; ++k2) {
        // W_M^{3072 n3 k2}: a uniform exponent (scalar-cache table reads)
        const float2 wk = tw_lookup(a.tw, 4ull * 3072u * n3 * static_cast<uint32_t>(k2));
        *reinterpret_cast<float2*>(outb + off) = cmul(z[k2], cmul(wo, wk));
        off += (pa_store_pos(0, 0, 1) - pa_store_pos(0, 0, 0)) * sizeof(float2);
      }
    }
  }
  }  // columns
  // block_sum's first barrier orders the scratch writes after the last reads of
  // the block; one partial per column slot (pass B sums all kAL3 of them)
  const double tot = block_sum<kAT>(static_cast<double>(fsum), reinterpret_cast<double*>(data));
  if (tid < kNC) a.partials[static_cast<size_t>(b) * kAL3 + kNC * blockIdx.x + tid] = tid == 0 ? tot : 0.0;
}

}  // namespace

std::string two_pass_selftest() {
  // pass A stores: a permutation of the column, and the inverse of tp_pos
  std::vector<uint8_t> seen(kAC, 0);
  for (uint32_t r = 0; r < 3; ++r)
    for (uint32_t k1 = 0; k1 < static_cast<uint32_t>(kALen); ++k1)
      for (uint32_t k2 = 0; k2 < 8; ++k2) {
        const uint32_t pos = pa_store_pos(r, k1, k2);
        if (pos >= kAC) return "pass A store position out of the column";
        if (seen[pos]++) return "pass A store position written twice";
        if (tp_pos(3u * (k1 + 1024u * k2) + r) != pos) return "tp_pos is not pass A's layout";
      }
  // LDS block: a_idx is a permutation of the 1024 x 8 block
  std::vector<uint8_t> lds(kALen * kACols, 0);
  for (int t = 0; t < kALen; ++t)
    for (int j = 0; j < kACols; ++j) {
      const int e = a_idx(t, j);
      if (e < 0 || e >= kALen * kACols || lds[e]++) return "a_idx is not a permutation";
    }
  // Stockham stages 16 x 8 x 8: each writes every row of a column once
  const int stages[3][2] = {{1, 16}, {16, 8}, {128, 8}};
  for (const auto& st : stages) {
    std::vector<uint8_t> rows(kALen, 0);
    for (int jp = 0; jp < kALen / st[1]; ++jp)
      for (int p = 0; p < st[1]; ++p) {
        const int row = a_stage_row(st[0], st[1], jp, p);
        if (row < 0 || row >= kALen || rows[row]++) return "Stockham stage rows";
      }
  }
  // pass B tiles: every row a workgroup loads maps into the column
  for (uint32_t blk = 0; blk < (kAC / 2 + 24) / 8; ++blk)
    for (uint32_t s = 0; s < 64; ++s) {
      const uint32_t cs = blk * 8 + (s % 32);
      const uint32_t row = s < 32 ? cs : (kAC - cs) % kAC;
      if (tp_pos(row < kAC ? row : 0) >= kAC) return "pass B row outside the column";
    }
  return "";
}

bool two_pass_supported(const FFTPlan3& plan, uint32_t n_unpadded) {
  return plan.L1 * plan.L2 == kAC && plan.L3 == kAL3 && plan.L2 * plan.L3 == kAL2L3 &&
         2ull * (kAC / 3) * kAL3 >= n_unpadded;
}

hipError_t launch_pass_a(const FFTPlan3& plan, const PassAArgs& a, int batch, hipStream_t s) {
  if (!two_pass_supported(plan, a.n_unpadded)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(pass_a_kernel, dim3(kAL3 / kNC, batch), dim3(kAT), 0, s, a);
  return hipGetLastError();
}

}  // namespace hipk
}  // namespace brp
