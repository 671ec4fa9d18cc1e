// Workgroup-level FFT building blocks for gfx950.
//
// A workgroup transforms NCOL independent sequences of length L that live in
// LDS. Each stage is a Stockham radix-R step (natural-order output, no bit
// reversal): butterfly j reads elements j + q*L/R, applies the stage twiddle
// W_{Ns*R}^{(j mod Ns) q}, does an R-point DFT in registers and writes element
// (j/Ns)*Ns*R + (j mod Ns) + q*Ns. Stage twiddles come from a per-length LDS
// table W_L^e (filled once per workgroup), so no transcendental is evaluated in
// the inner loop.
//
// Two LDS layouts:
//   column layout (ROWMAJOR=false): element (r, c) at r*NCOL + c, lanes walk c
//     fastest -> the strided "column" passes read/write 8*NCOL contiguous bytes
//     per row of the global array (128 B for NCOL=16).
//   row layout    (ROWMAJOR=true):  element (r, c) at c*(L+1) + r, lanes walk r
//     fastest -> the contiguous "row" pass streams whole rows.
#pragma once

#include "hip_common.hpp"

namespace brp {
namespace hipk {

// ---------------------------------------------------------------- radix DFTs
// Forward DFTs (kernel exp(-2 pi i / R)), in place on registers.
template <int R>
struct Dft;

template <>
struct Dft<2> {
  static __device__ __forceinline__ void run(float2* v) {
    const float2 a = v[0], b = v[1];
    v[0] = cadd(a, b);
    v[1] = csub(a, b);
  }
};

template <>
struct Dft<3> {
  static __device__ __forceinline__ void run(float2* v) {
    const float s = 0.86602540378443864676f;  // sin(2pi/3)
    const float2 t1 = cadd(v[1], v[2]);
    const float2 t2 = cfma(-0.5f, t1, v[0]);
    const float2 d = csub(v[1], v[2]);
    v[0] = cadd(v[0], t1);
    v[1] = add_mi(t2, d, s);  // t2 + (-i) s d
    v[2] = sub_mi(t2, d, s);
  }
};

template <>
struct Dft<4> {
  static __device__ __forceinline__ void run(float2* v) {
    const float2 a0 = cadd(v[0], v[2]), a1 = csub(v[0], v[2]);
    const float2 b0 = cadd(v[1], v[3]), d = csub(v[1], v[3]);
    v[0] = cadd(a0, b0);
    v[1] = add_mi(a1, d);  // a1 + (-i) d
    v[2] = csub(a0, b0);
    v[3] = sub_mi(a1, d);
  }
};

template <>
struct Dft<5> {
  static __device__ __forceinline__ void run(float2* v) {
    const float c1 = 0.30901699437494742410f, c2 = -0.80901699437494742410f;
    const float s1 = 0.95105651629515357212f, s2 = 0.58778525229247312917f;
    const float2 a1 = cadd(v[1], v[4]), a2 = cadd(v[2], v[3]);
    const float2 b1 = csub(v[1], v[4]), b2 = csub(v[2], v[3]);
    const float2 x0 = v[0];
    const float2 p1 = cfma(c2, a2, cfma(c1, a1, x0));
    const float2 p2 = cfma(c1, a2, cfma(c2, a1, x0));
    const float2 q1 = cfma(s2, b2, cscale(b1, s1));   // (-i) q1 is added below
    const float2 q2 = cfma(-s1, b2, cscale(b1, s2));
    v[0] = cadd(x0, cadd(a1, a2));
    v[1] = add_mi(p1, q1);
    v[4] = sub_mi(p1, q1);
    v[2] = add_mi(p2, q2);
    v[3] = sub_mi(p2, q2);
  }
};

// radix 7 (lengths 7 * 16 * 2^a: N = 7 * 2^k paddings such as -P 3.5 take
// the three-pass path instead of the chirp-z transform): pairs v_j +- v_{7-j},
// X_k = p_k - i q_k and X_{7-k} = p_k + i q_k with p_k = v_0 + sum_j cos(2 pi jk/7) a_j,
// q_k = sum_j sin(2 pi jk/7) b_j
template <>
struct Dft<7> {
  static __device__ __forceinline__ void run(float2* v) {
    const float c1 = 0.62348980185873353053f, c2 = -0.22252093395631440429f, c3 = -0.90096886790241912624f;
    const float s1 = 0.78183148246802980871f, s2 = 0.97492791218182360702f, s3 = 0.43388373911755812048f;
    const float2 a1 = cadd(v[1], v[6]), a2 = cadd(v[2], v[5]), a3 = cadd(v[3], v[4]);
    const float2 b1 = csub(v[1], v[6]), b2 = csub(v[2], v[5]), b3 = csub(v[3], v[4]);
    const float2 x0 = v[0];
    const float2 p1 = cfma(c3, a3, cfma(c2, a2, cfma(c1, a1, x0)));
    const float2 p2 = cfma(c1, a3, cfma(c3, a2, cfma(c2, a1, x0)));
    const float2 p3 = cfma(c2, a3, cfma(c1, a2, cfma(c3, a1, x0)));
    const float2 q1 = cfma(s3, b3, cfma(s2, b2, cscale(b1, s1)));
    const float2 q2 = cfma(-s1, b3, cfma(-s3, b2, cscale(b1, s2)));
    const float2 q3 = cfma(s2, b3, cfma(-s1, b2, cscale(b1, s3)));
    v[0] = cadd(x0, cadd(cadd(a1, a2), a3));
    v[1] = add_mi(p1, q1);
    v[6] = sub_mi(p1, q1);
    v[2] = add_mi(p2, q2);
    v[5] = sub_mi(p2, q2);
    v[3] = add_mi(p3, q3);
    v[4] = sub_mi(p3, q3);
  }
};

template <>
struct Dft<8> {
  static __device__ __forceinline__ void run(float2* v) {
    const float r = 0.70710678118654752440f;
    float2 e[4] = {v[0], v[2], v[4], v[6]};
    float2 o[4] = {v[1], v[3], v[5], v[7]};
    Dft<4>::run(e);
    Dft<4>::run(o);
    // o[k] *= W8^k: W8 = r (1 - i), W8^2 = -i, W8^3 = r (-1 - i)
    o[1] = cscale(add_mi(o[1], o[1]), r);                       // r (o.x + o.y, o.y - o.x)
    o[2] = mul_mi(o[2]);
    o[3] = cscale(add_mi(make_float2(-o[3].x, -o[3].y), o[3]), r);  // r (o.y - o.x, -o.x - o.y)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[k] = cadd(e[k], o[k]);
      v[k + 4] = csub(e[k], o[k]);
    }
  }
};

template <>
struct Dft<16> {
  static __device__ __forceinline__ void run(float2* v) {
    // x[a + 4b]: DFT4 over b for each a, twiddle W16^{a k1}, DFT4 over a
    float2 u[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      float2 t[4] = {v[a], v[a + 4], v[a + 8], v[a + 12]};
      Dft<4>::run(t);
#pragma unroll
      for (int k = 0; k < 4; ++k) u[a][k] = t[k];
    }
    const float c1 = 0.92387953251128675613f, s1 = 0.38268343236508977173f;
    const float r = 0.70710678118654752440f;
    // W16^1, W16^2, W16^3, W16^4 = -i, W16^6, W16^9
    const float2 w1 = make_float2(c1, -s1), w2 = make_float2(r, -r), w3 = make_float2(s1, -c1);
    const float2 w6 = make_float2(-r, -r), w9 = make_float2(-c1, s1);
    u[1][1] = cmul(u[1][1], w1);
    u[1][2] = cmul(u[1][2], w2);
    u[1][3] = cmul(u[1][3], w3);
    u[2][1] = cmul(u[2][1], w2);
    u[2][2] = mul_mi(u[2][2]);
    u[2][3] = cmul(u[2][3], w6);
    u[3][1] = cmul(u[3][1], w3);
    u[3][2] = cmul(u[3][2], w6);
    u[3][3] = cmul(u[3][3], w9);
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1) {
      float2 t[4] = {u[0][k1], u[1][k1], u[2][k1], u[3][k1]};
      Dft<4>::run(t);
#pragma unroll
      for (int k2 = 0; k2 < 4; ++k2) v[k1 + 4 * k2] = t[k2];
    }
  }
};

// ------------------------------------------------------------ block FFT core
// Row layout: one pad element every 16 (r + r/16) and a row pitch == 16 (mod 32)
// keep both the radix-16 scatter (stride-16 writes of a 16-lane group) and the
// two-row reads of a 32-lane group bank-conflict free.
template <int L>
constexpr int row_pitch() {
  return (L + L / 16) + ((16 - (L + L / 16) % 32) + 32) % 32;
}

template <int L, int NCOL, int TPC, bool ROWMAJOR>
struct BlockLayout {
  static constexpr int kThreads = NCOL * TPC;
  static constexpr int kPitch = row_pitch<L>();
  // Row layout: slot c also gets a skew of 4 (c / 2) elements. Slot pairs
  // (2i, 2i+1) keep the pitch == 16 (mod 32) spacing that the two-row stage
  // accesses need, while the 8 slots a wave touches in the untangle (lanes
  // walk slots, then 4 consecutive bins) start on 8 distinct 8-dword bank
  // groups instead of 2 (measured: 25 % of pass 3's LDS cycles were conflicts).
  static constexpr int kLds = ROWMAJOR ? NCOL * kPitch + 4 * (NCOL / 2) : L * NCOL;  // float2 elements
  __device__ __forceinline__ static int idx(int r, int c) {
    return ROWMAJOR ? c * kPitch + 4 * (c >> 1) + r + (r >> 4) : r * NCOL + c;
  }
  __device__ __forceinline__ static void coords(int tid, int& c, int& tj) {
    if (ROWMAJOR) {
      tj = tid % TPC;
      c = tid / TPC;
    } else {
      c = tid % NCOL;
      tj = tid / NCOL;
    }
  }
};

// Stage twiddle table W_L^e (e < L) stored at e + e/16 (kTwPad<L> entries) so the
// stride-q reads of a radix-16 stage do not collide on LDS banks. The host
// precomputes it in exactly this order; kernels copy it contiguously to LDS.
template <int L>
constexpr int kTwPad = L + L / 16 + 1;

// 8-byte LDS load kept a ds_read_b64: left to itself the load-store optimiser
// pairs neighbouring loads into ds_read2_b64, which the LDS services as 4 x 16
// lanes on 32 banks -- twice the cycles of two ds_read_b64, and the row
// layout's skews assume the 64-bank b64 mapping (cdna_hip_programming.md §2)
__device__ __forceinline__ float2 lds_ld64(const float2* p) {
  using f2 = float __attribute__((ext_vector_type(2)));
  const f2 v = *(const volatile f2 __attribute__((address_space(3)))*)(p);
  return make_float2(v.x, v.y);
}

// Row passes (pass 3): the last radix-16 stage (Ns = L / 16) reads its
// twiddles W_L^{jm q} from a q-major block [q - 1][jm] appended to the padded
// stage table, so the 16 butterflies of a row read 16 consecutive entries.
// (From the padded table the stride-jm reads collided: 44 extra LDS cycles per
// wave, all of pass 3's bank conflicts in profiles/pmc_bytes_pruned_hs_r2.txt.)
template <int L>
constexpr int kTwRowExtra = 15 * (L / 16);

// One Stockham stage LDS -> LDS (in place, two barriers).
template <int L, int NCOL, int TPC, bool ROWMAJOR, int R, int Ns>
__device__ __forceinline__ void block_stage(float2* lds, const float2* tw_lds) {
  using Lay = BlockLayout<L, NCOL, TPC, ROWMAJOR>;
  constexpr int kBf = L / R;                       // butterflies per column
  constexpr int kNb = (kBf + TPC - 1) / TPC;       // butterflies per thread
  constexpr bool kQMajor = ROWMAJOR && Ns > 1 && Ns * R == L;
  static_assert(!kQMajor || R == 16, "row passes end in a radix-16 stage");
  int c, tj;
  Lay::coords(threadIdx.x, c, tj);
  float2 v[kNb][R];
#pragma unroll
  for (int u = 0; u < kNb; ++u) {
    const int j = tj + u * TPC;
    if (kBf % TPC == 0 || j < kBf) {
#pragma unroll
      for (int q = 0; q < R; ++q) {
        const float2* p = &lds[Lay::idx(j + q * kBf, c)];
        v[u][q] = ROWMAJOR ? lds_ld64(p) : *p;
      }
      if (Ns > 1) {
        const int jm = j % Ns;
#pragma unroll
        for (int q = 1; q < R; ++q) {
          float2 w;
          if constexpr (kQMajor) {
            w = lds_ld64(&tw_lds[kTwPad<L> + (q - 1) * Ns + jm]);
          } else {
            const int e = (jm * q * (L / (Ns * R))) % L;
            w = tw_lds[e + (e >> 4)];  // padded: stride-q reads hit distinct banks
          }
          v[u][q] = cmul(v[u][q], w);
        }
      }
      Dft<R>::run(v[u]);
    }
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < kNb; ++u) {
    const int j = tj + u * TPC;
    if (kBf % TPC == 0 || j < kBf) {
      const int base = (j / Ns) * Ns * R + (j % Ns);
#pragma unroll
      for (int q = 0; q < R; ++q) lds[Lay::idx(base + q * Ns, c)] = v[u][q];
    }
  }
  __syncthreads();
}

// First stage (Ns = 1, no twiddles) of radix R on data whose rows >= L/R are
// zero: the DFT of (x, 0, ..., 0) is (x, ..., x), so the stage copies row j to
// rows R j .. R j + R - 1 (the zero rows are never read).
template <int L, int NCOL, int TPC, bool ROWMAJOR, int R>
__device__ __forceinline__ void block_stage_replicate(float2* lds) {
  using Lay = BlockLayout<L, NCOL, TPC, ROWMAJOR>;
  constexpr int kBf = L / R;
  constexpr int kNb = (kBf + TPC - 1) / TPC;
  int c, tj;
  Lay::coords(threadIdx.x, c, tj);
  float2 v[kNb];
#pragma unroll
  for (int u = 0; u < kNb; ++u) {
    const int j = tj + u * TPC;
    if (kBf % TPC == 0 || j < kBf) v[u] = lds[Lay::idx(j, c)];
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < kNb; ++u) {
    const int j = tj + u * TPC;
    if (kBf % TPC == 0 || j < kBf) {
#pragma unroll
      for (int q = 0; q < R; ++q) lds[Lay::idx(R * j + q, c)] = v[u];
    }
  }
  __syncthreads();
}

template <int L, int NCOL, int TPC, bool ROWMAJOR, int Ns, int... Rs>
struct BlockStages;

template <int L, int NCOL, int TPC, bool ROWMAJOR, int Ns>
struct BlockStages<L, NCOL, TPC, ROWMAJOR, Ns> {
  static __device__ __forceinline__ void run(float2*, const float2*) {}
};

template <int L, int NCOL, int TPC, bool ROWMAJOR, int Ns, int R, int... Rest>
struct BlockStages<L, NCOL, TPC, ROWMAJOR, Ns, R, Rest...> {
  static __device__ __forceinline__ void run(float2* lds, const float2* tw) {
    block_stage<L, NCOL, TPC, ROWMAJOR, R, Ns>(lds, tw);
    BlockStages<L, NCOL, TPC, ROWMAJOR, Ns * R, Rest...>::run(lds, tw);
  }
};

template <int... Rs>
struct Product;
template <>
struct Product<> {
  static constexpr int value = 1;
};
template <int R, int... Rest>
struct Product<R, Rest...> {
  static constexpr int value = R * Product<Rest...>::value;
};

// Radix decomposition for each supported sub-FFT length.
template <int L>
struct Radices;
template <> struct Radices<16> { template <template <int...> class F> using apply = F<16>; };
template <> struct Radices<32> { template <template <int...> class F> using apply = F<2, 16>; };
template <> struct Radices<48> { template <template <int...> class F> using apply = F<3, 16>; };
template <> struct Radices<64> { template <template <int...> class F> using apply = F<4, 16>; };
template <> struct Radices<80> { template <template <int...> class F> using apply = F<5, 16>; };
template <> struct Radices<112> { template <template <int...> class F> using apply = F<7, 16>; };
template <> struct Radices<224> { template <template <int...> class F> using apply = F<2, 7, 16>; };
template <> struct Radices<448> { template <template <int...> class F> using apply = F<4, 7, 16>; };
template <> struct Radices<96> { template <template <int...> class F> using apply = F<3, 2, 16>; };
template <> struct Radices<128> { template <template <int...> class F> using apply = F<8, 16>; };
template <> struct Radices<144> { template <template <int...> class F> using apply = F<3, 3, 16>; };
template <> struct Radices<160> { template <template <int...> class F> using apply = F<5, 2, 16>; };
template <> struct Radices<192> { template <template <int...> class F> using apply = F<3, 4, 16>; };
template <> struct Radices<240> { template <template <int...> class F> using apply = F<3, 5, 16>; };
template <> struct Radices<288> { template <template <int...> class F> using apply = F<3, 3, 2, 16>; };
template <> struct Radices<256> { template <template <int...> class F> using apply = F<16, 16>; };
template <> struct Radices<320> { template <template <int...> class F> using apply = F<5, 4, 16>; };
template <> struct Radices<384> { template <template <int...> class F> using apply = F<3, 8, 16>; };
template <> struct Radices<512> { template <template <int...> class F> using apply = F<2, 16, 16>; };

template <int L, int NCOL, int TPC, bool ROWMAJOR>
struct BlockFFT {
  template <int... Rs>
  struct Impl {
    static_assert(Product<Rs...>::value == L, "radix list must multiply to L");
    static __device__ __forceinline__ void run(float2* lds, const float2* tw) {
      BlockStages<L, NCOL, TPC, ROWMAJOR, 1, Rs...>::run(lds, tw);
    }
  };
  static __device__ __forceinline__ void run(float2* lds, const float2* tw) {
    Radices<L>::template apply<Impl>::run(lds, tw);
  }
  // rows >= L / R0 are zero (R0 = first radix): replicate instead of stage 1
  template <int R0, int... Rs>
  struct ImplPruned {
    static constexpr int kFirst = R0;
    static __device__ __forceinline__ void run(float2* lds, const float2* tw) {
      block_stage_replicate<L, NCOL, TPC, ROWMAJOR, R0>(lds);
      BlockStages<L, NCOL, TPC, ROWMAJOR, R0, Rs...>::run(lds, tw);
    }
  };
  static constexpr int kFirstRadix = Radices<L>::template apply<ImplPruned>::kFirst;
  static __device__ __forceinline__ void run_pruned(float2* lds, const float2* tw) {
    Radices<L>::template apply<ImplPruned>::run(lds, tw);
  }
  // stages 2.. only: the caller has done stage 1 (radix kFirstRadix, Ns = 1)
  // in registers and written its Stockham output to LDS
  template <int R0, int... Rs>
  struct ImplRest {
    static __device__ __forceinline__ void run(float2* lds, const float2* tw) {
      BlockStages<L, NCOL, TPC, ROWMAJOR, R0, Rs...>::run(lds, tw);
    }
  };
  static __device__ __forceinline__ void run_rest(float2* lds, const float2* tw) {
    Radices<L>::template apply<ImplRest>::run(lds, tw);
  }
};

// ------------------------------------------------------------ shared helpers
// block-wide deterministic sum of one double per thread (result valid in all threads)
template <int NT>
__device__ __forceinline__ double block_sum(double v, double* scratch) {
  v = wave_sum(v);
  const int w = threadIdx.x / kWave;
  constexpr int kWaves = (NT + kWave - 1) / kWave;
  __syncthreads();
  if ((threadIdx.x % kWave) == 0) scratch[w] = v;
  __syncthreads();
  double t = 0.0;
#pragma unroll
  for (int i = 0; i < kWaves; ++i) t += scratch[i];
  __syncthreads();
  return t;
}

// a * conj(b) as packed operations (the conjugate's sign folds into the
// instruction instead of a v_xor)
__device__ __forceinline__ float2 cmulc(float2 a, float2 b) {
  const f2v av = vec(a), bv = vec(b);
  const f2v bc = {bv.x, -bv.y};
  return unvec(__builtin_elementwise_fma(av.yy, bv.yx, av.xx * bc));  // as cmul
}

// X_k of the real FFT from Z_k, Z_{M-k} of the packed complex FFT and w = W_N^k:
// e = (Z_k + conj Z_{M-k}) / 2, o = (Z_k - conj Z_{M-k}) / 2, X_k = e - i w o
__device__ __forceinline__ float2 untangle_w(float2 zk, float2 zmk, float2 w) {
  const f2v h = 0.5f * vec(zk), m = vec(zmk);
  const float2 e = unvec(__builtin_elementwise_fma(m, f2v{0.5f, -0.5f}, h));
  const float2 o = unvec(__builtin_elementwise_fma(m, f2v{-0.5f, 0.5f}, h));
  return add_mi(e, cmul(w, o));
}
// the mirror bin M - k from the same pair: untangle_w(Z_{M-k}, Z_k, W_N^{M-k})
// with W_N^{M-k} = -conj(W_N^k): e' + i conj(w) o'
__device__ __forceinline__ float2 untangle_wm(float2 zmk, float2 zk, float2 w) {
  const f2v h = 0.5f * vec(zmk), m = vec(zk);
  const float2 e = unvec(__builtin_elementwise_fma(m, f2v{0.5f, -0.5f}, h));
  const float2 o = unvec(__builtin_elementwise_fma(m, f2v{-0.5f, 0.5f}, h));
  return sub_mi(e, cmulc(o, w));
}

// FFT of the padding indicator 1[m >= n_s] (m < N) at bin k in [1, N/2]:
// S_k = -(sin(pi n_s k / N) / sin(pi k / N)) * exp(-i pi (n_s - 1) k / N),
// from ta = W_2N^{n_s k}, tk = W_2N^k, tc = W_2N^{(n_s-1) k}.
__device__ __forceinline__ float2 padding_spectrum_t(float2 ta, float2 tk, float2 tc) {
  const float ratio = ta.y / tk.y;
  return make_float2(-ratio * tc.x, -ratio * tc.y);
}

// multiply by (-i)^q
__device__ __forceinline__ float2 rot_mi(float2 a, uint32_t q) {
  switch (q & 3u) {
    case 0: return a;
    case 1: return make_float2(a.y, -a.x);
    case 2: return make_float2(-a.x, -a.y);
    default: return make_float2(-a.y, a.x);
  }
}


template <int L>
__device__ __forceinline__ void copy_stage_twiddles(float2* tw_lds, const float2* __restrict__ st) {
  for (int e = threadIdx.x; e < kTwPad<L>; e += blockDim.x) tw_lds[e] = BRP_LD(&st[e]);
}

// row-pass stage table: padded W_L^e, then the last stage's q-major block
// (host: stage_table_rows in hip_engine.cpp)
template <int L>
__device__ __forceinline__ void copy_row_twiddles(float2* tw_lds, const float2* __restrict__ st) {
  for (int e = threadIdx.x; e < kTwPad<L> + kTwRowExtra<L>; e += blockDim.x) tw_lds[e] = BRP_LD(&st[e]);
}

}  // namespace hipk
}  // namespace brp
