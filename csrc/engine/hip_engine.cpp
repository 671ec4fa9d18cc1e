// MI355X backend: device state of one work unit and batched template processing.
//
// Per batch of B templates one HIP graph replays
//   H2D params -> H2D thresholds -> memset counters -> n_steps -> FFT pass 1
//   (fused resampling) -> pass 2 -> pass 3 (untangle + power spectrum) ->
//   harmonic sum + compaction -> D2H counters + first candidate slots
// with a single host synchronisation per batch. The reference issues ~11
// launches, 5 blocking transfers and up to ~6 MB of device->host copies per
// template (cuda/app/demod_binary_cuda.cu:416-965, demod_binary_hs_cuda.cu:302-677).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <tuple>
#include <mutex>
#include <string>
#include <unordered_map>

#include "../core/errors.hpp"
#include "../core/fault.hpp"
#include "../core/trace.hpp"
#include "../core/gsl_compat.hpp"
#include "../core/cpu_backend.hpp"
#include "../core/log.hpp"
#include "../core/rngmed.hpp"
#include "../core/wisdom.hpp"
#include "../hip/bluestein_kernels.hpp"
#include "../hip/fft_kernels.hpp"
#include "../hip/hs_kernels.hpp"
#include "../hip/resample_kernels.hpp"
#include "../hip/whiten_kernels.hpp"
#include "backend.hpp"
#include "hip_engine.hpp"

namespace brp {

using hipk::TemplateDev;

namespace {
// W_{L2 L3} as lo[256] x hi[1024] (build_tables): L2 L3 <= 2^18, so that the
// chirp-z convolution of the longest odd N (P = 10 at 2^22 samples: L >= 84 M)
// has a plan (512 x 2^17 = 67 M was the limit before round 5)
constexpr uint64_t kMaxL2L3 = 256ull * 1024;
const uint32_t kPlanP3[] = {256, 320, 192, 160, 128, 96, 64};
const uint32_t kPlanP12[] = {512, 448, 384, 320, 288, 256, 240, 224, 192, 160, 144, 128, 112, 96, 80, 64, 48, 32, 16};
}  // namespace

// Chirp-z transform of length Mb (bluestein_kernels.hpp): the smallest length
// L >= 2 Mb - 1 the three-pass FFT factors. The products L1 L2 L3 of the
// compiled lengths are dense (16 * 2^a 3^b 5^c 7^d), so L stays within ~10 % of
// the minimum.
bool make_bluestein_plan(uint32_t Mb, FFTPlan3& plan) {
  const uint64_t need = 2ull * Mb - 1;
  std::vector<uint64_t> lens;
  // BRP_BS_L3 (A/B): only convolution lengths whose plan has this row length
  const uint32_t want_l3 = std::getenv("BRP_BS_L3") ? static_cast<uint32_t>(std::atoi(std::getenv("BRP_BS_L3"))) : 0;
  for (uint32_t L3 : kPlanP3)
    for (uint32_t L1 : kPlanP12)
      for (uint32_t L2 : kPlanP12) {
        if (L2 > L1 || static_cast<uint64_t>(L2) * L3 > kMaxL2L3 || !hipk::pass12_length_supported(L2)) continue;
        const uint64_t L = static_cast<uint64_t>(L1) * L2 * L3;
        if (L >= need && L < (1ull << 31)) lens.push_back(L);
      }
  if (lens.empty()) return false;
  std::sort(lens.begin(), lens.end());
  lens.erase(std::unique(lens.begin(), lens.end()), lens.end());
  // BRP_BS_PLAN=L1xL2xL3 (A/B): that factorisation when it covers the length
  // and meets the enumeration's constraints (L2 <= L1, the pass-2 twiddle
  // table's L2 L3 <= kMaxL2L3, a length below 2^31); otherwise ignored
  if (const char* e = std::getenv("BRP_BS_PLAN")) {
    unsigned a1 = 0, a2 = 0, a3 = 0;
    const bool parsed = std::sscanf(e, "%ux%ux%u", &a1, &a2, &a3) == 3;
    const uint64_t len = static_cast<uint64_t>(a1) * a2 * a3;
    if (parsed && len >= need && len < (1ull << 31) && a2 <= a1 && static_cast<uint64_t>(a2) * a3 <= kMaxL2L3 &&
        hipk::pass12_length_supported(a1) && hipk::pass12_length_supported(a2) && hipk::pass3_length_supported(a3)) {
      plan = FFTPlan3();
      plan.M = static_cast<uint32_t>(len);
      plan.L1 = a1;
      plan.L2 = a2;
      plan.L3 = a3;
      plan.ncol1 = plan.ncol2 = 16;
      plan.rows3 = 8;
      return true;
    }
    log_message(LOG_WARN, true, "BRP_BS_PLAN=%s ignored: not a supported factorisation of a length >= %llu.\n", e,
                static_cast<unsigned long long>(need));
  }
  if (want_l3) {
    for (uint64_t L : lens)
      if (make_fft_plan(static_cast<uint32_t>(L), plan) && plan.L3 == want_l3 && hipk::chirp_rev_supported(plan))
        return true;
  }
  // Among the lengths up to 20 % above the shortest, the lowest modelled cost
  // of a plan that runs the transposed convolution (hipk::chirp_rev_supported):
  // L times 1.15 when the row length L3 takes three LDS stages (96, 160, 192,
  // 320) rather than two (64, 128, 256). Measured in one call (round 5):
  // -P 2.9 3 566 templates/s over 256 x 192 x 256 against 3 107 over the
  // 2.4 % shorter 240 x 160 x 320; -P 2.7 3 402 vs 3 219 (2.9 % longer).
  double best_cost = 0.0;
  uint64_t best = 0;
  for (uint64_t L : lens) {
    if (L > lens.front() + lens.front() / 5) break;
    if (!make_fft_plan(static_cast<uint32_t>(L), plan) || !hipk::chirp_rev_supported(plan)) continue;
    const bool two_stage = plan.L3 == 64 || plan.L3 == 128 || plan.L3 == 256;
    const double cost = static_cast<double>(L) * (two_stage ? 1.0 : 1.15);
    if (best == 0 || cost < best_cost) {
      best = L;
      best_cost = cost;
    }
  }
  return make_fft_plan(static_cast<uint32_t>(best ? best : lens.front()), plan);
}

bool make_fft_plan(uint32_t M, FFTPlan3& plan) {
  plan = FFTPlan3();
  // preference: long pass-3 rows (contiguous PS writes), then balanced L1 >= L2
  const auto& p3 = kPlanP3;
  const auto& p12 = kPlanP12;
  for (uint32_t L3 : p3) {
    if (M % L3) continue;
    const uint32_t R = M / L3;
    uint32_t best1 = 0, best2 = 0;
    for (uint32_t L1 : p12) {
      if (R % L1) continue;
      const uint32_t L2 = R / L1;
      if (!hipk::pass12_length_supported(L2)) continue;
      if (L1 < L2) continue;
      if (static_cast<uint64_t>(L2) * L3 > kMaxL2L3) continue;  // pass-2 twiddle table (256 x 1024)
      if (!best1 || (L1 - L2) < (best1 - best2)) {
        best1 = L1;
        best2 = L2;
      }
    }
    if (best1) {
      plan.M = M;
      plan.L1 = best1;
      plan.L2 = best2;
      plan.L3 = L3;
      plan.ncol1 = plan.ncol2 = 16;
      plan.rows3 = 8;
      return true;
    }
  }
  return false;
}

namespace {

// BRP_FAULT=hip_oom: every device allocation fails; hip_oom:N: the first N
// succeed (so the first pipeline sets up and a later one fails)
std::atomic<long> g_device_allocs{0};  // device allocations of this process (fault tests)

bool fault_device_alloc() {
  const long k = g_device_allocs.fetch_add(1);
  std::string param;
  if (!fault_enabled("hip_oom", &param)) return false;
  const long ok = param.empty() ? 0 : std::atol(param.c_str());
  return k >= ok;
}

template <typename T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  // fine: fine-grained device memory the host can read and write in place
  // (over the PCIe BAR) -- used for the per-batch parameters and results
  // checked build (hipk::checked_build()): a guard zone behind the requested
  // bytes, and the allocation in the registry the device-side checks read
  int alloc(size_t count, bool fine = false) {
    release();
    if (count == 0) return 0;
    const size_t bytes = count * sizeof(T), total = bytes + hipk::chk_guard_bytes();
    const hipError_t e = fine ? hipExtMallocWithFlags(reinterpret_cast<void**>(&p), total, hipDeviceMallocFinegrained)
                              : hipMalloc(&p, total);
    if (fault_device_alloc() || e != hipSuccess) {
      if (e == hipSuccess) (void)hipFree(p);  // injected failure
      else (void)hipGetLastError();
      p = nullptr;
      log_message(LOG_ERROR, true, "Couldn't allocate %zu bytes of device memory!\n", bytes);
      return RADPUL_HIP_MEM_ALLOC_DEVICE;
    }
    if (total > bytes) {
      if (hipk::chk_fill_guard(p, bytes) != hipSuccess) (void)hipGetLastError();
      hipk::chk_register(p, bytes, total);
    }
    n = count;
    return 0;
  }
  void release() {
    if (p) {
      hipk::chk_unregister(p);
      (void)hipFree(p);
    }
    p = nullptr;
    n = 0;
  }
  ~DevBuf() { release(); }
};

template <typename T>
struct PinnedBuf {
  T* p = nullptr;
  size_t n = 0;
  bool pageable = false;
  // Pinned first; if the runtime refuses (locked-memory limits), fall back to
  // pageable memory like the reference's HS host buffers
  // (cuda/app/demod_binary_hs_cuda.cu:207-219): copies then stage through the
  // runtime's own pinned bounce buffers, slower but correct.
  int alloc(size_t count) {
    release();
    if (count == 0) return 0;
    if (fault_enabled("pinned_fail") || hipHostMalloc(&p, count * sizeof(T), hipHostMallocDefault) != hipSuccess) {
      p = static_cast<T*>(std::malloc(count * sizeof(T)));
      if (!p) return RADPUL_HIP_MEM_ALLOC_HOST;
      pageable = true;
      log_message(LOG_WARN, true, "Couldn't allocate %zu bytes of pinned host memory, using pageable memory.\n",
                  count * sizeof(T));
    }
    n = count;
    return 0;
  }
  void release() {
    if (p && n) {  // n == 0: a non-owning view
      if (pageable)
        std::free(p);
      else
        (void)hipHostFree(p);
    }
    p = nullptr;
    n = 0;
    pageable = false;
  }
  // at least `count` elements (contents not kept)
  int reserve(size_t count) { return count <= n ? 0 : alloc(count); }
  ~PinnedBuf() { release(); }
};

// Synchronous copy on the engine's own stream. A plain hipMemcpy goes through
// the null stream, whose first use creates one more hardware queue: 7.5-8.3 ms
// of start-up on MI355X (tools/experiments/startup/, profiles/README.md round 3).
// Every host <-> device copy of the engine: the host side is pinned memory
// (or a host view of fine-grained device memory), never pageable memory; the
// checked build verifies that (hipk::chk_host_copy).
hipError_t memcpy_async(void* dst, const void* src, size_t bytes, hipMemcpyKind kind, hipStream_t s) {
  if (kind == hipMemcpyHostToDevice) hipk::chk_host_copy(src, bytes);
  else if (kind == hipMemcpyDeviceToHost) hipk::chk_host_copy(dst, bytes);
  return hipMemcpyAsync(dst, src, bytes, kind, s);
}

// page-locked host memory the runtime knows (hipHostMalloc, hipHostRegister):
// copies may read / write it directly
bool host_pinned(const void* p) {
  hipPointerAttribute_t at{};
  if (hipPointerGetAttributes(&at, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return at.type == hipMemoryTypeHost;
}

hipError_t copy_sync(void* dst, const void* src, size_t bytes, hipMemcpyKind kind, hipStream_t s) {
  const hipError_t e = memcpy_async(dst, src, bytes, kind, s);
  if (e != hipSuccess) return e;
  return hipStreamSynchronize(s);
}

// A fine-grained device allocation the host may read and write in place: on
// a large-BAR device (all MI355X platforms) ROCm maps device memory into the
// host address space at the same address. Checked with a host-written pattern
// read back through a device copy.
void* host_view(int device, void* p, size_t bytes, hipStream_t s, PinnedBuf<uint8_t>& scratch) {
  int large_bar = 0;
  if (hipDeviceGetAttribute(&large_bar, hipDeviceAttributeIsLargeBar, device) != hipSuccess) return nullptr;
  hipPointerAttribute_t at{};
  if (hipPointerGetAttributes(&at, p) != hipSuccess) return nullptr;
  void* h = at.hostPointer != nullptr ? at.hostPointer : p;
  log_message(LOG_DEBUG, true, "fine-grained buffer %p: large BAR %d, host pointer %p -> %p\n", p, large_bar,
              at.hostPointer, h);
  if (!large_bar) return nullptr;
  std::vector<uint8_t> pat(bytes);
  for (size_t i = 0; i < bytes; ++i) pat[i] = static_cast<uint8_t>(i * 37u + 11u);
  std::memcpy(h, pat.data(), bytes);
  std::atomic_thread_fence(std::memory_order_seq_cst);
  // read back through the engine's pinned stage (one allocation for all checks)
  if (scratch.reserve(bytes) || copy_sync(scratch.p, p, bytes, hipMemcpyDeviceToHost, s) != hipSuccess) return nullptr;
  return std::memcmp(pat.data(), scratch.p, bytes) == 0 ? h : nullptr;
}

// W_{2N}^j = exp(-i pi j / N) as a two-level float table
void build_twiddles(uint64_t period, std::vector<float2>& hi, std::vector<float2>& lo) {
  const uint32_t nlo = 1u << hipk::kTwLoBits;
  const uint64_t nhi = (period + nlo - 1) / nlo + 1;
  hi.resize(nhi);
  lo.resize(nlo);
  const long double pi = 3.14159265358979323846264338327950288L;
  auto w = [&](uint64_t j) {
    j %= period;
    const long double a = -2.0L * pi * static_cast<long double>(j) / static_cast<long double>(period);
    return make_float2(static_cast<float>(cosl(a)), static_cast<float>(sinl(a)));
  };
  for (uint64_t i = 0; i < nhi; ++i) hi[i] = w(i * nlo);
  for (uint32_t j = 0; j < nlo; ++j) lo[j] = w(j);
}

// exp(-2 pi i num/den) with exact integer reduction
float2 root(uint64_t num, uint64_t den) {
  num %= den;
  const long double pi = 3.14159265358979323846264338327950288L;
  const long double a = -2.0L * pi * static_cast<long double>(num) / static_cast<long double>(den);
  return make_float2(static_cast<float>(cosl(a)), static_cast<float>(sinl(a)));
}

std::vector<float2> stage_table(uint32_t L) {
  std::vector<float2> t(L + L / 16 + 1, make_float2(0.f, 0.f));
  for (uint32_t e = 0; e < L; ++e) t[e + (e >> 4)] = root(e, L);
  return t;
}

// row passes (pass 3): the padded table, then W_L^{jm q} as [q - 1][jm] for the
// last radix-16 stage, jm < L / 16 (fft_block.hpp, copy_row_twiddles)
std::vector<float2> stage_table_rows(uint32_t L) {
  std::vector<float2> t = stage_table(L);
  for (uint32_t q = 1; q < 16; ++q)
    for (uint32_t jm = 0; jm < L / 16; ++jm) t.push_back(root(static_cast<uint64_t>(jm) * q, L));
  return t;
}

// Host-built twiddle tables of one plan (single rounding from long double).
// Every pipeline of a process (and every pass of a task) uses the same plan,
// so they are computed once: ~80 000 long-double sin/cos per plan.
struct HostTables {
  std::vector<float2> st1, st2, st3, p1, p2col, p2lo, p2hi, p3;
};

const HostTables& host_tables(const FFTPlan3& plan) {
  static std::mutex mu;
  static std::map<std::tuple<uint32_t, uint32_t, uint32_t>, std::unique_ptr<HostTables>> cache;
  std::lock_guard<std::mutex> lk(mu);
  auto& slot = cache[std::make_tuple(plan.L1, plan.L2, plan.L3)];
  if (slot) return *slot;
  auto h = std::make_unique<HostTables>();
  const uint32_t L1 = plan.L1, L2 = plan.L2, L3 = plan.L3, M = plan.M;
  const uint64_t L2L3 = static_cast<uint64_t>(L2) * L3;
  h->st1 = stage_table(L1);
  h->st2 = stage_table(L2);
  h->st3 = stage_table_rows(L3);
  h->p1.resize(static_cast<size_t>(L2) * L1);
  for (uint32_t n2 = 0; n2 < L2; ++n2)
    for (uint32_t k1 = 0; k1 < L1; ++k1)
      h->p1[n2 * L1 + k1] = root(static_cast<uint64_t>(n2) * k1, static_cast<uint64_t>(L1) * L2);
  h->p2col.assign(static_cast<size_t>(L1) * L3, make_float2(0, 0));
  for (uint32_t k1 = 0; k1 < L1; ++k1)
    for (uint32_t n3 = 0; n3 < L3; ++n3) h->p2col[k1 * L3 + n3] = root(static_cast<uint64_t>(n3) * k1, M);
  h->p2lo.assign(256, make_float2(0, 0));
  for (uint32_t i = 0; i < 256; ++i) h->p2lo[i] = root(i, L2L3);
  h->p2hi.assign(1024, make_float2(0, 0));
  for (uint32_t i = 0; i < 1024 && 256ull * i < L2L3; ++i) h->p2hi[i] = root(256ull * i, L2L3);
  // pass 3: W_{4 L3}^j = hi[j >> 5] * lo[j & 31], stored as [lo 32 | hi 4 L3 / 32]
  h->p3.assign(32 + 4ull * L3 / 32, make_float2(0, 0));
  for (uint32_t i = 0; i < 32; ++i) h->p3[i] = root(i, 4ull * L3);
  for (uint32_t m = 0; m < 4 * L3 / 32; ++m) h->p3[32 + m] = root(32ull * m, 4ull * L3);
  slot = std::move(h);
  return *slot;
}

// W_period two-level tables, cached per period like the plan tables
const std::pair<std::vector<float2>, std::vector<float2>>& twiddles_cached(uint64_t period) {
  static std::mutex mu;
  static std::map<uint64_t, std::unique_ptr<std::pair<std::vector<float2>, std::vector<float2>>>> cache;
  std::lock_guard<std::mutex> lk(mu);
  auto& slot = cache[period];
  if (!slot) {
    slot = std::make_unique<std::pair<std::vector<float2>, std::vector<float2>>>();
    build_twiddles(period, slot->first, slot->second);
  }
  return *slot;
}

}  // namespace

// launch groups per submitted batch (Impl::serial): measured in profiles/README.md (round 3)
constexpr int kDefaultSerial = 4;

struct HipEngine::Impl {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;  // views of the current batch I/O slot
  int batch = 4;                // templates per kernel launch (grid.y), each with its own FFT buffers
  // Templates of one submitted batch run `serial` launch groups of `batch`
  // templates back to back through the same FFT buffers: one completion event
  // per submitted batch instead of one per group (an event record costs the
  // stream ~7 us of idle GPU time; profiles/README.md round 3). BRP_SERIAL.
  int serial = 1;
  int batch_req = 4, serial_req = 1;  // as requested at init (setup adapts them to the geometry)
  int slot_cap() const { return batch * serial; }  // templates per submitted batch
  hipEvent_t prev_done = nullptr;  // completion event of the last completed batch (device-time statistics)
  uint32_t key_base = 0;        // template index of the current launch group within its batch
  bool group_reset = true;      // the current launch group zeroes the batch's candidate counter
  uint32_t cap = 1u << 20;      // candidate slots per batch (all templates and levels; BRP_HS_CAP)
  uint32_t bin_bits = 23;       // candidate key layout (hs_pack) of the geometry
  // Bounded output (hipk::launch_harmonic_sum_select): per template and level
  // only the values >= the 100th largest are emitted. Switched on when a
  // batch's list overflows (that batch is re-run), off again once a batch's
  // above-threshold count would fit the list comfortably. BRP_HS_SELECT=1: always.
  bool select_mode = false;
  bool select_forced = false;
  DevBuf<float> sel_dense;
  DevBuf<uint32_t> sel_hist, sel_state;
  uint32_t dense_stride = 0;
  int ensure_select() {
    const size_t rows = static_cast<size_t>(batch) * 5;
    int rc;
    if (sel_dense.n < rows * dense_stride && (rc = sel_dense.alloc(rows * dense_stride))) return rc;
    if (sel_hist.n < rows * hipk::kHsSelBins && (rc = sel_hist.alloc(rows * hipk::kHsSelBins))) return rc;
    if (sel_state.n < rows * 4 && (rc = sel_state.alloc(rows * 4))) return rc;
    return 0;
  }
  uint32_t kcopy = 1024;        // slots copied back with every batch (more: second copy)
  // results in place (fg_out): longer lists are DMA-copied instead of read over
  // the PCIe BAR (uncached host reads; config 4 measured 12.8k vs 17.4k pairs/s
  // reading every list in place). BRP_FG_INPLACE_MAX, at most kcopy.
  uint32_t inplace_max = 1024;

  SearchGeometry g;
  FFTPlan3 plan;
  // Chirp-z path for lengths the three-pass FFT does not factor: `plan` is
  // then the length-L plan of the convolution, the DFT has length bs_Mb
  // (N/2 for even N, N for odd N); bluestein_kernels.hpp
  bool bs = false;
  // odd N: two templates per chirp-z transform (real / imaginary part,
  // P1_CHIRP1_PAIR), half the convolution work per template. BRP_BS_PAIR=0: one
  bool bs_pair = false;
  int bs_trans(int nb) const { return bs_pair ? (nb + 1) / 2 : nb; }
  uint32_t bs_Mb = 0;
  DevBuf<float2> bs_a;          // [batch][L] chirp-in / convolution spectrum / A
  DevBuf<float2> bs_h;          // [L] FFT_L of the wrapped conjugate chirp
  // template transforms as the transposed convolution (bluestein_kernels.hpp:
  // pass3_mid, reverse passes 2 and 1) with H in row layout; BRP_BS_REV=0:
  // the natural-order form (pass3_cplx, a second forward transform)
  bool bs_rev = false;
  DevBuf<float2> bs_hp;         // [L] H in the row layout
  DevBuf<float2> bs_chirp_hi, bs_chirp_lo;  // W_{2 Mb}
  bool ready = false;
  uint32_t num_cus = 256;
  std::string arch;             // gcnArchName (plan-wisdom lookup)
  bool ps_fp16 = false;         // config 5: fp16 power spectrum between pass 3 and the harmonic sum
  uint32_t persist_per_cu = 4;  // persistent FFT passes: workgroups per CU (BRP_PERSIST, 0 = off)
  uint32_t ps_stride = 0;
  int32_t i_start = 0;
  // per-batch parameters / candidate results in fine-grained device memory the
  // host writes / reads directly, instead of two small copies per batch
  // (each a runtime blit kernel on the GPU); BRP_FG=in|out|both|0
  bool fg_in = false, fg_out = false;

  DevBuf<float> series;
  DevBuf<uint8_t> wu_packed;    // staging of the WU payload (setup_packed)
  // read-only series of a sibling pipeline on the same device (adopt_series):
  // one copy for all pipelines keeps the Infinity-Cache footprint down
  const float* shared_series = nullptr;
  const float* series_in() const { return shared_series != nullptr ? shared_series : series.p; }
  // Generation of this engine's own series buffer: bumped whenever it is
  // reallocated, rewritten or freed. An engine reading it in place holds the
  // token (which outlives this engine) and the generation it adopted, and
  // refuses to launch once they differ (the source was set up again, whitened
  // another WU or destroyed before the reader was set up again).
  std::shared_ptr<std::atomic<uint64_t>> series_token = std::make_shared<std::atomic<uint64_t>>(0);
  std::shared_ptr<std::atomic<uint64_t>> adopted_token;
  uint64_t adopted_gen = 0;
  void bump_series() { series_token->fetch_add(1); }
  bool shared_series_valid() const {
    return shared_series == nullptr || (adopted_token && adopted_token->load() == adopted_gen);
  }
  // back to the engine's own series (before anything writes it)
  void own_series() {
    bump_series();
    if (shared_series == nullptr) return;
    shared_series = nullptr;
    adopted_token.reset();
    for (auto& kv : graphs) (void)hipGraphExecDestroy(kv.second);  // captured series pointer changed
    graphs.clear();
  }
  DevBuf<float2> buf;           // [batch][M]
  DevBuf<uint8_t> w_rmed;       // wide-window running-median scratch (whitening)
  DevBuf<float> ps;             // [batch][ps_stride]
  DevBuf<float> pyr;            // [batch][hs_pyr_stride(ps_stride)]: 8-bin maxima of the spectrum (pruned HS)
  bool hs_prune = true;         // pruned harmonic sum (BRP_HS_FULL=1: every block exactly)
  int hs_cell_shift = 3;        // its bound cells: 8 bins (BRP_HS_CELL=4: 4 bins, tighter bounds but
                                // 44 KB LDS / 125 VGPRs per workgroup: 16.4-16.7k vs 15.6-15.8k templates/s)
  bool hs_xcd = false;          // pruned HS: contiguous block ranges per XCD (BRP_HS_XCD=1)
  bool lds_pass1 = false;       // resampling pass 1 on the LDS-staged kernel (BRP_P1_LDS=1, A/B)
  bool mid_waves = false;       // pass3_mid: whole-wave workgroups of 16 / 32 rows (BRP_MID_WAVES=1, A/B)
  // 8-bin bound cells of the own bins written by pass 3 (pass3_kernel CELLS),
  // hs_cells_kernel only for the mirror half; BRP_P3_CELLS=1 (A/B, default off:
  // profiles/README.md round 6)
  bool p3_cells = false;
  bool fused_cells() const { return p3_cells && hs_prune && hs_cell_shift == 3 && !bs; }
  // 8-bin cells per thread of the fp32 cell kernel (BRP_HS_CELLS_CPT: 1 or 4)
  uint32_t hs_cells_cpt = 1;
  bool hs_direct = true;        // bounds read straight from global memory (BRP_HS_DIRECT=0: LDS-staged;
                                // +2 % fp32, +3 % config 5 in one call, profiles/README.md round 3)
  DevBuf<double> partials;      // [batch][wg1]
  DevBuf<double> delta;         // [batch] mean-padding correction
  // Per-batch I/O, double-buffered so that a pipeline can keep two batches in
  // flight on its stream (submit / complete): the next batch's parameters are
  // written and its graph launched while the previous one runs, so the GPU
  // does not wait on the host between batches. The FFT, spectrum and cell
  // buffers stay single: the stream orders the two batches.
  //   in:    thresholds | templates (ONE host->device copy, or written in place)
  //   cands: [1 + cap] count | (packed key, power) entries
  struct BatchIO {
    DevBuf<uint8_t> in;
    PinnedBuf<uint8_t> h_in;
    DevBuf<uint2> cands;
    PinnedBuf<uint2> h_cands;
    uint8_t* h_in_p = nullptr;  // host view of the parameters (pinned copy or `in` itself)
    uint2* h_cands_p = nullptr;  // host view of the results (pinned copy or `cands` itself)
    hipEvent_t ev0 = nullptr, ev1 = nullptr;  // ev0: stage benchmark only; ev1: the batch's completion
    int nb = 0;
    bool pending = false;
    bool sel = false;  // submitted with the bounded output (select_mode)
  };
  static constexpr int kIoSlots = 3;  // I/O slots; BRP_INFLIGHT picks how many are used (default 2)
  BatchIO io[kIoSlots];
  int io_cur = 0, io_next = 0, io_head = 0;
  // views of slot io_cur, used by enqueue_stage / capture and the test hooks
  struct { uint8_t* p = nullptr; } in, h_in;
  struct { TemplateDev* p = nullptr; } tmpl;
  struct { float* p = nullptr; } thr;
  struct { uint2* p = nullptr; } cands;
  void select_io(int i) {
    io_cur = i;
    BatchIO& o = io[i];
    in.p = o.in.p;
    h_in.p = o.h_in_p;
    thr.p = reinterpret_cast<float*>(o.in.p);
    tmpl.p = reinterpret_cast<TemplateDev*>(o.in.p + thr_bytes);
    h_thr.p = reinterpret_cast<float*>(o.h_in_p);
    h_tmpl.p = reinterpret_cast<TemplateDev*>(o.h_in_p + thr_bytes);
    cands.p = o.cands.p;
    h_cands.p = o.h_cands_p;
    ev0 = o.ev0;
    ev1 = o.ev1;
  }
  bool io_busy() const {
    for (const BatchIO& o : io)
      if (o.pending) return true;
    return false;
  }
  DevBuf<float2> tw_hi, tw_lo;
  DevBuf<float2> w_spec, w_z;   // whitening scratch: half spectrum, packed inverse input
  DevBuf<float> w_psw, w_med;   // whitening scratch: power spectrum, running median
  DevBuf<uint32_t> w_zbins;     // whitening: zapped bins and their noise
  DevBuf<float2> w_znoise;
  // Whitening that keeps its result on the device returns without waiting:
  // the pipelines that read the series order themselves after it with
  // ev_w1 (adopt_series), so the host's prepare / launch work overlaps the
  // whitening kernels. The host noise arrays stay alive until ev_w1 has passed.
  PinnedBuf<uint32_t> w_zb_host;  // pinned: the copies are truly asynchronous
  PinnedBuf<float2> w_zn_host;
  // Host copies of the engine go through its own pinned buffers, never through
  // the runtime's pageable-memory path (which pins the caller's pages for each
  // copy and has the device write them: the one device fault seen on a test
  // box, round 5, was such a copy; profiles/fault_r6.txt): `stage` bounces the
  // large one-off copies (series, spectra, cells, tables) in chunks, `list_host`
  // receives candidate lists too long to read in place.
  PinnedBuf<uint8_t> stage;
  PinnedBuf<uint2> list_host;
  static constexpr size_t kStageChunk = 8u << 20;
  hipError_t copy_out(void* dst, const void* src, size_t bytes) {
    if (bytes == 0) return hipSuccess;
    if (host_pinned(dst)) return copy_sync(dst, src, bytes, hipMemcpyDeviceToHost, stream);  // caller's pinned buffer
    if (stage.reserve(std::min(bytes, kStageChunk))) return hipErrorOutOfMemory;
    for (size_t off = 0; off < bytes; off += kStageChunk) {
      const size_t nb = std::min(kStageChunk, bytes - off);
      hipError_t e = memcpy_async(stage.p, static_cast<const uint8_t*>(src) + off, nb, hipMemcpyDeviceToHost, stream);
      if (e == hipSuccess) e = hipStreamSynchronize(stream);
      if (e != hipSuccess) return e;
      std::memcpy(static_cast<uint8_t*>(dst) + off, stage.p, nb);
    }
    return hipSuccess;
  }
  hipError_t copy_in(void* dst, const void* src, size_t bytes) {
    if (bytes == 0) return hipSuccess;
    // a registered source (the WU buffers search.cpp / multi.cpp page-lock) is read directly
    if (host_pinned(src)) return copy_sync(dst, src, bytes, hipMemcpyHostToDevice, stream);
    if (stage.reserve(std::min(bytes, kStageChunk))) return hipErrorOutOfMemory;
    for (size_t off = 0; off < bytes; off += kStageChunk) {
      const size_t nb = std::min(kStageChunk, bytes - off);
      hipError_t e = hipStreamSynchronize(stream);  // the stage's previous chunk has been read
      if (e != hipSuccess) return e;
      std::memcpy(stage.p, static_cast<const uint8_t*>(src) + off, nb);
      e = memcpy_async(static_cast<uint8_t*>(dst) + off, stage.p, nb, hipMemcpyHostToDevice, stream);
      if (e != hipSuccess) return e;
    }
    return hipStreamSynchronize(stream);
  }
  hipEvent_t ev_w0 = nullptr, ev_w1 = nullptr, ev_adopt = nullptr;
  bool w_pending = false;       // ev_w0 / ev_w1 of an asynchronous whitening not yet accounted
  // whitening device time of a finished asynchronous whitening into the stats
  void settle_whiten(bool wait) {
    if (!w_pending) return;
    if (!wait && hipEventQuery(ev_w1) != hipSuccess) {
      (void)hipGetLastError();
      return;
    }
    (void)hipEventSynchronize(ev_w1);
    float ms = 0;
    if (hipEventElapsedTime(&ms, ev_w0, ev_w1) == hipSuccess) st.whiten_ms += ms;
    w_pending = false;
  }
  DevBuf<float2> t_st1, t_st2, t_st3, t_p1, t_p2col, t_p2lo, t_p2hi, t_p3;

  struct { TemplateDev* p = nullptr; } h_tmpl;
  struct { float* p = nullptr; } h_thr;
  struct { uint2* p = nullptr; } h_cands;  // [1 + kcopy]
  size_t thr_bytes = 64;        // thresholds area at the start of `in`: [batch][kHsThrStride] floats
  uint32_t slots = 1;           // work-unit slots of the series buffer (multi-WU batching)
  std::vector<float> mu0s;      // per-slot padding offset

  std::map<int, hipGraphExec_t> graphs;  // key: (batch size * kIoSlots + I/O slot) * 2 + select mode
  BackendStats st;

  hipk::FFTTables tables() const {
    hipk::FFTTables t;
    t.st1 = t_st1.p;
    t.st2 = t_st2.p;
    t.st3 = t_st3.p;
    t.p1 = t_p1.p;
    t.p2col = t_p2col.p;
    t.p2lo = t_p2lo.p;
    t.p2hi = t_p2hi.p;
    t.p3 = t_p3.p;
    return t;
  }

  int upload(DevBuf<float2>& d, const std::vector<float2>& h) {
    int rc = d.alloc(h.size());
    if (rc) return rc;
    if (copy_in(d.p, h.data(), h.size() * sizeof(float2)) != hipSuccess) return RADPUL_HIP_MEM_COPY_HOST_DEVICE;
    return 0;
  }

  int build_tables() {
    const HostTables& h = host_tables(plan);
    int rc;
    if ((rc = upload(t_st1, h.st1)) || (rc = upload(t_st2, h.st2)) || (rc = upload(t_st3, h.st3)) ||
        (rc = upload(t_p1, h.p1)) || (rc = upload(t_p2col, h.p2col)) || (rc = upload(t_p2lo, h.p2lo)) ||
        (rc = upload(t_p2hi, h.p2hi)) || (rc = upload(t_p3, h.p3)))
      return rc;
    return 0;
  }

  hipk::TwiddleTable twt() const {
    hipk::TwiddleTable t;
    t.hi = tw_hi.p;
    t.lo = tw_lo.p;
    t.period = 2ull * g.nsamples;  // W_2N (= W_{4M} of the packed transform)
    t.inv_period = 1.0 / static_cast<double>(t.period);
    return t;
  }
  hipk::TwiddleTable chirpt() const {
    hipk::TwiddleTable t;
    t.hi = bs_chirp_hi.p;
    t.lo = bs_chirp_lo.p;
    t.period = 2ull * bs_Mb;
    t.inv_period = 1.0 / static_cast<double>(t.period);
    return t;
  }

  // ---- chirp-z path
  // y (bs_a) -> FFT_L -> * H, conj (bs_a) -> FFT_L -> conj * w / L = A (bs_a)
  // (whitening; the template path starts from the series: bs_template_in)
  hipError_t bs_convolve(int nb) {
    hipError_t e = bs_round(nb, 0);
    return e == hipSuccess ? bs_round(nb, 1) : e;
  }
  hipError_t bs_round(int nb, int round) {
    return bs_fft(nb, round == 0 ? hipk::C3_MULCONJ : hipk::C3_CHIRP, bs_a.p);
  }
  // one length-L transform of bs_a (passes 1, 2 and the epilogue of `mode` into out)
  hipError_t bs_fft(int nb, hipk::Pass3CplxMode mode, float2* out) {
    hipk::Pass1Args a1{};
    a1.out = buf.p;
    a1.L2L3 = plan.L2 * plan.L3;
    a1.L3 = plan.L3;
    a1.tw = twt();
    a1.tb = tables();
    a1.cplx_in = bs_a.p;
    hipError_t e = hipk::launch_pass1(plan, hipk::P1_COMPLEX, a1, nb, stream);
    return e == hipSuccess ? bs_fft_rest(nb, mode, out, 0) : e;
  }
  // passes 2 and 3 of a length-L transform in buf; n_partials > 0: pass 2
  // also reduces pass 1's template partial sums (delta)
  hipError_t bs_fft_rest(int nb, hipk::Pass3CplxMode mode, float2* out, uint32_t n_partials, uint32_t tpt = 1,
                         uint32_t n_tmpl = 0) {
    const hipk::TwiddleTable tw = twt();
    const bool reduce_delta = n_partials > 0;
    hipError_t e;
    hipk::Pass2Args a2{};
    a2.buf = buf.p;
    a2.L1 = plan.L1;
    a2.L2L3 = plan.L2 * plan.L3;
    a2.L3 = plan.L3;
    a2.tw = tw;
    a2.tb = tables();
    if (reduce_delta) {
      a2.partials = partials.p;
      a2.n_partials = n_partials;
      a2.tmpl = tmpl.p;
      a2.delta = delta.p;
      a2.tpt = tpt;
      a2.n_tmpl = n_tmpl;
    }
    if ((e = hipk::launch_pass2(plan, a2, nb, stream)) != hipSuccess) return e;
    hipk::Pass3CplxArgs a3{};
    a3.buf = buf.p;
    a3.L1 = plan.L1;
    a3.L2 = plan.L2;
    a3.L3 = plan.L3;
    a3.C = plan.L1 * plan.L2;
    a3.M = plan.M;
    a3.tb = tables();
    a3.out = out;
    a3.out_stride = plan.M;
    a3.h = bs_h.p;
    a3.chirp = chirpt();
    a3.n_out = bs_Mb;
    a3.scale = static_cast<float>(1.0 / static_cast<double>(plan.M));
    return hipk::launch_pass3_cplx(plan, mode, a3, nb, stream);
  }
  // H = FFT_L of the wrapped conjugate chirp (once per plan)
  hipError_t bs_make_h() {
    hipk::BsInArgs a = bs_in();
    hipError_t e = hipk::launch_bs_chirp_in(hipk::BS_IN_HCHIRP, a, 1, nullptr, stream);
    return e == hipSuccess ? bs_fft(1, hipk::C3_PLAIN, bs_h.p) : e;
  }
  hipk::BsInArgs bs_in() const {
    hipk::BsInArgs a{};
    a.y = bs_a.p;
    a.L = plan.M;
    a.Mb = bs_Mb;
    a.nsamples = g.nsamples;
    a.chirp = chirpt();
    return a;
  }
  // template spectra of a batch of nb templates: pass 1 of the first
  // convolution transform straight from the series (resampling, centring,
  // chirp: P1_CHIRP*), its passes 2 and 3 (* H), the second transform, the
  // power spectrum (bins k < limit into ps_out [nb][stride]); bs_trans(nb)
  // transforms (paired templates for odd N)
  hipError_t bs_template_in(int nb, uint32_t* reset) {
    hipk::Pass1Args a1{};
    a1.out = buf.p;
    a1.L2L3 = plan.L2 * plan.L3;
    a1.L3 = plan.L3;
    a1.tw = twt();
    a1.tb = tables();
    a1.series = series_in();
    a1.n_unpadded = g.n_unpadded;
    a1.tmpl = tmpl.p;
    a1.partials = partials.p;
    a1.reset = reset;
    a1.chirp = chirpt();
    a1.Mb = bs_Mb;
    a1.n_tmpl = static_cast<uint32_t>(nb);
    const hipk::Pass1Mode m = bs_pair ? hipk::P1_CHIRP1_PAIR : (bs_Mb == g.nsamples ? hipk::P1_CHIRP1 : hipk::P1_CHIRP2);
    return hipk::launch_pass1(plan, m, a1, bs_trans(nb), stream);
  }
  hipError_t bs_template_round0(int nb) {
    if (bs_rev) {  // forward pass 2 (+ delta), then the middle: rows * H, conj, inverse rows, in place
      hipk::Pass2Args a2 = bs_pass2_args(plan.wg1(), bs_pair ? 2u : 1u, static_cast<uint32_t>(nb));
      hipError_t e = hipk::launch_pass2(plan, a2, bs_trans(nb), stream);
      if (e != hipSuccess) return e;
      hipk::Pass3MidArgs am{};
      am.buf = buf.p;
      am.hp = bs_hp.p;
      am.L1 = plan.L1;
      am.L2 = plan.L2;
      am.L3 = plan.L3;
      am.tb = tables();
      am.whole_waves = mid_waves;
      return hipk::launch_pass3_mid(plan, am, bs_trans(nb), stream);
    }
    return bs_fft_rest(bs_trans(nb), hipk::C3_MULCONJ, bs_a.p, plan.wg1(), bs_pair ? 2u : 1u, static_cast<uint32_t>(nb));
  }
  // the inverse transform's columns in transposed order: reverse pass 2, then
  // pass 1 with the final chirp into bs_a (A, n < Mb)
  hipError_t bs_template_round1(int nb) {
    if (!bs_rev) return bs_round(bs_trans(nb), 1);
    hipk::Pass2Args a2 = bs_pass2_args(0, 1, 0);
    a2.rev = true;
    hipError_t e = hipk::launch_pass2(plan, a2, bs_trans(nb), stream);
    if (e != hipSuccess) return e;
    hipk::Pass1Args a1{};
    a1.out = bs_a.p;
    a1.L2L3 = plan.L2 * plan.L3;
    a1.L3 = plan.L3;
    a1.tw = twt();
    a1.tb = tables();
    a1.cplx_in = buf.p;
    a1.chirp = chirpt();
    a1.Mb = bs_Mb;
    a1.scale = static_cast<float>(1.0 / static_cast<double>(plan.M));
    return hipk::launch_pass1(plan, hipk::P1_REV_CHIRP, a1, bs_trans(nb), stream);
  }
  hipk::Pass2Args bs_pass2_args(uint32_t n_partials, uint32_t tpt, uint32_t n_tmpl) {
    hipk::Pass2Args a2{};
    a2.buf = buf.p;
    a2.L1 = plan.L1;
    a2.L2L3 = plan.L2 * plan.L3;
    a2.L3 = plan.L3;
    a2.tw = twt();
    a2.tb = tables();
    if (n_partials > 0) {
      a2.partials = partials.p;
      a2.n_partials = n_partials;
      a2.tmpl = tmpl.p;
      a2.delta = delta.p;
      a2.tpt = tpt;
      a2.n_tmpl = n_tmpl;
    }
    return a2;
  }
  hipError_t bs_template_power(int nb, float* ps_out, _Float16* ps16_out, uint32_t stride, uint32_t limit) {
    hipk::BsPowerArgs ap{};
    ap.A = bs_a.p;
    ap.L = plan.M;
    ap.Mb = bs_Mb;
    ap.nsamples = g.nsamples;
    ap.tw = twt();
    ap.limit = limit;
    ap.ps = ps_out;
    ap.ps16 = ps16_out;
    ap.ps_stride = stride;
    ap.norm = static_cast<float>(1.0 / g.nsamples);
    ap.tmpl = tmpl.p;
    ap.delta = delta.p;
    ap.pair = bs_pair;
    ap.n_tmpl = static_cast<uint32_t>(nb);
    return hipk::launch_bs_power(ap, bs_trans(nb), stream);
  }
  hipError_t bs_template_spectra(int nb, float* ps_out, _Float16* ps16_out, uint32_t stride, uint32_t limit) {
    hipError_t e = bs_template_in(nb, nullptr);
    if (e == hipSuccess) e = bs_template_round0(nb);
    if (e == hipSuccess) e = bs_template_round1(nb);
    return e == hipSuccess ? bs_template_power(nb, ps_out, ps16_out, stride, limit) : e;
  }

  ~Impl() {
    bump_series();  // readers of this series must not launch any more
    for (hipEvent_t e : {ev_w0, ev_w1, ev_adopt})
      if (e) (void)hipEventDestroy(e);
    for (auto& kv : graphs) (void)hipGraphExecDestroy(kv.second);
    for (BatchIO& o : io) {
      if (o.ev0) (void)hipEventDestroy(o.ev0);
      if (o.ev1) (void)hipEventDestroy(o.ev1);
    }
    if (stream) (void)hipStreamDestroy(stream);
  }

  // Template transform, pass 1 (fused resampling gather). `reset`: the
  // batch's candidate counter to zero.
  hipError_t fft_pass1(int nb, uint32_t* reset) {
    const hipk::TwiddleTable tw = twt();
    hipk::Pass1Args a1{};
    a1.out = buf.p;
    a1.L2L3 = plan.L2 * plan.L3;
    a1.L3 = plan.L3;
    a1.tw = tw;
    a1.tb = tables();
    a1.series = series_in();
    a1.n_unpadded = g.n_unpadded;
    a1.tmpl = tmpl.p;
    a1.partials = partials.p;
    a1.reset = reset;
    a1.lds_pass1 = lds_pass1;
    return hipk::launch_pass1(plan, hipk::P1_RESAMPLE, a1, nb, stream);
  }
  hipError_t fft_pass2(int nb) {
    hipk::Pass2Args a2{};
    a2.buf = buf.p;
    a2.L1 = plan.L1;
    a2.L2L3 = plan.L2 * plan.L3;
    a2.L3 = plan.L3;
    a2.tw = twt();
    a2.tb = tables();
    a2.partials = partials.p;
    a2.n_partials = plan.wg1();
    a2.tmpl = tmpl.p;
    a2.delta = delta.p;
    return hipk::launch_pass2(plan, a2, nb, stream);
  }
  // row pass + untangle + power spectrum into out[b * stride + k], k < limit;
  // with_cells: also the pruned harmonic sum's 8-bin bound cells of the own
  // (low-residue) bins (pyr), so that the harmonic sum re-reads only half the
  // spectrum for the others
  hipError_t fft_pass3(int nb, float* out, _Float16* out16, uint32_t stride, uint32_t limit, bool with_cells = false) {
    hipk::Pass3Args a3{};
    a3.buf = buf.p;
    a3.L1 = plan.L1;
    a3.L2 = plan.L2;
    a3.L3 = plan.L3;
    a3.C = plan.L1 * plan.L2;
    a3.M = plan.M;
    a3.tw = twt();
    a3.tb = tables();
    a3.limit = limit;
    a3.ps = out;
    a3.ps16 = out16;
    a3.ps_stride = stride;
    a3.norm = static_cast<float>(1.0 / g.nsamples);
    a3.tmpl = tmpl.p;
    a3.delta = delta.p;
    if (with_cells) {
      a3.cells = pyr.p;
      a3.cells_stride = hipk::hs_pyr_stride(ps_stride);
      a3.n_cells = (ps_stride >> 3) + 8;  // what hs_cells_kernel writes (8-bin cells)
    }
    return hipk::launch_pass3(plan, hipk::P3_POWER, a3, nb, stream);
  }

  // Pipeline stages of one batch; the whole sequence is captured into a graph.
  enum Stage { kPrologue = 0, kPass1, kPass2, kPass3, kHarmonic, kEpilogue, kNumStages };

  hipError_t enqueue_stage(int st, int nb) {
    hipError_t e = hipSuccess;
    switch (st) {
      case kPrologue:
        // n_steps comes with the parameters (host bracketed search); pass 1
        // zeroes the batch's candidate counter
        if (fg_in) return hipSuccess;  // the host wrote `in` directly
        return memcpy_async(in.p, h_in.p, thr_bytes + sizeof(TemplateDev) * nb, hipMemcpyHostToDevice, stream);
      case kPass1:
        if (bs) return bs_template_in(nb, group_reset ? &cands.p[0].x : nullptr);
        return fft_pass1(nb, group_reset ? &cands.p[0].x : nullptr);
      case kPass2:
        if (bs) return bs_template_round0(nb);
        return fft_pass2(nb);
      case kPass3: {
        if (bs) {
          const hipError_t e3 = bs_template_round1(nb);
          if (e3 != hipSuccess) return e3;
          return bs_template_power(nb, ps.p, ps_fp16 ? reinterpret_cast<_Float16*>(ps.p) : nullptr, ps_stride,
                                   std::min(g.harmonic_idx_hi, g.fft_size));
        }
        return fft_pass3(nb, ps.p, ps_fp16 ? reinterpret_cast<_Float16*>(ps.p) : nullptr, ps_stride,
                         std::min(g.harmonic_idx_hi, g.fft_size), fused_cells());
      }
      case kHarmonic: {
        hipk::HSArgs ah{};
        ah.mode = ps_fp16 ? hipk::HS_F16 : hipk::HS_F32;
        ah.ps = ps.p;
        ah.ps16 = ps_fp16 ? reinterpret_cast<const _Float16*>(ps.p) : nullptr;
        ah.ps_stride = ps_stride;
        ah.w2 = g.window_2;
        ah.fhi = g.fundamental_idx_hi;
        ah.hhi = std::min(g.harmonic_idx_hi, g.fft_size);
        ah.i_start = i_start;
        ah.thr = thr.p;
        ah.list = cands.p;
        ah.cap = cap;
        ah.prune = hs_prune;
        ah.cell_shift = hs_cell_shift;
        ah.direct = hs_direct && hs_cell_shift == 3;
        ah.xcd = hs_xcd;
        ah.pyr = pyr.p;
        ah.pyr_stride = hipk::hs_pyr_stride(ps_stride);
        ah.cells_ready = !bs && fused_cells();  // pass 3 wrote the own-bin cells
        ah.cells_cpt = hs_cells_cpt;
        ah.row_c = plan.L1 * plan.L2;
        ah.row_l = plan.L3;
        ah.key_base = key_base;
        ah.bin_bits = bin_bits;
        if (select_mode) {
          hipk::HsSelectArgs sa{};
          sa.dense = sel_dense.p;
          sa.dense_stride = dense_stride;
          sa.hist = sel_hist.p;
          sa.state = sel_state.p;
          sa.k = kCandPerLevel;
          return hipk::launch_harmonic_sum_select(ah, sa, nb, stream);
        }
        return hipk::launch_harmonic_sum(ah, nb, stream);
      }
      case kEpilogue:
        if (fg_out) return hipSuccess;  // the host reads `cands` directly
        return memcpy_async(h_cands.p, cands.p, sizeof(uint2) * (1 + kcopy), hipMemcpyDeviceToHost, stream);
      default: return hipErrorInvalidValue;
    }
  }

  // Enqueue the whole per-batch pipeline on `stream` (also used for capture):
  // launch groups of up to `batch` templates back to back (passes 1-3 and the
  // harmonic sum each), the parameter upload before the first group and the
  // candidate read-back after the last. Each group reads its templates and
  // thresholds at its offset in the batch's I/O slot and appends to the
  // batch's one candidate list (keys carry the template's index in the batch).
  hipError_t enqueue(int nb) {
    TemplateDev* const tmpl0 = tmpl.p;
    float* const thr0 = thr.p;
    hipError_t e = enqueue_stage(kPrologue, nb);
    // bounded output: list[0].y counts the batch's above-threshold values
    if (e == hipSuccess && select_mode) e = hipMemsetAsync(cands.p, 0, sizeof(uint2), stream);
    for (int g0 = 0; e == hipSuccess && g0 < nb; g0 += batch) {
      const int ng = std::min(batch, nb - g0);
      tmpl.p = tmpl0 + g0;
      thr.p = thr0 + static_cast<size_t>(g0) * hipk::kHsThrStride;
      key_base = static_cast<uint32_t>(g0);
      group_reset = g0 == 0;
      for (int st = kPass1; e == hipSuccess && st <= kHarmonic; ++st) e = enqueue_stage(st, ng);
    }
    tmpl.p = tmpl0;
    thr.p = thr0;
    key_base = 0;
    group_reset = true;
    return e == hipSuccess ? enqueue_stage(kEpilogue, nb) : e;
  }
};

HipEngine::HipEngine() : impl_(new Impl) {}
HipEngine::~HipEngine() {
  if (impl_ && impl_->stream) (void)hipStreamSynchronize(impl_->stream);
  delete impl_;
}

namespace {
bool g_blocking_sync = false;

// Standalone device choice when neither -D, BOINC's gpu_device_num nor
// BRP_DEVICE names one: the device with the highest CU count x clock
// (reference findBestFreeDevice, cuda/app/cuda_utilities.c:96-237, by GFLOPS;
// device properties only, no context is created on the other GPUs).
int best_device(int ndev) {
  int best = 0;
  double best_score = -1.0;
  for (int d = 0; d < ndev; ++d) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, d) != hipSuccess) continue;
    const double score = static_cast<double>(prop.multiProcessorCount) * prop.clockRate;
    if (score > best_score) {
      best_score = score;
      best = d;
    }
  }
  return best;
}

void log_mem_status(int device, const char* when) {
  size_t free_b = 0, total_b = 0;
  if (hipMemGetInfo(&free_b, &total_b) == hipSuccess)
    log_message(LOG_DEBUG, true, "HIP device #%d global memory %s: %.1f MB free of %.1f MB\n", device, when,
                free_b / 1e6, total_b / 1e6);
}
}  // namespace

void hip_set_blocking_sync(bool on) { g_blocking_sync = on; }

void hip_prepare_host_tables(const SearchGeometry& g) {
  FFTPlan3 p;
  if (g.nsamples % 2 == 0 && make_fft_plan(g.nsamples / 2, p)) {
    (void)host_tables(p);
  } else {
    const uint32_t mb = g.nsamples % 2 ? g.nsamples : g.nsamples / 2;
    if (!make_bluestein_plan(mb, p)) return;
    (void)host_tables(p);
    (void)twiddles_cached(2ull * mb);
  }
  (void)twiddles_cached(2ull * g.nsamples);
}

void hip_runtime_warm_up() {
  int n = 0;
  (void)hipGetDeviceCount(&n);
  (void)hipGetLastError();
}

int hip_running_median(int device, const std::vector<float>& in, uint32_t W, std::vector<float>& out, int reps,
                       double* ms_per_call) {
  if (W == 0 || in.size() < W) return RADPUL_EVAL;
  BRP_HIP_CHECK(hipSetDevice(device < 0 ? 0 : device), RADPUL_HIP_DEVICE_SET);
  DevBuf<float> din, dout;
  DevBuf<uint8_t> scratch;
  int rc;
  const size_t n_out = in.size() - W + 1;
  if ((rc = din.alloc(in.size())) || (rc = dout.alloc(n_out))) return rc;
  bool wide = !hipk::running_median_supported(W);
  if (!wide && W > 3072) {  // the 128 KB LDS kernel needs a device with that much per workgroup
    int lds = 0;
    wide = hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerBlock, device < 0 ? 0 : device) != hipSuccess ||
           lds < 16384 * 8;
  }
  const uint32_t n_in = static_cast<uint32_t>(in.size());
  if (wide && (rc = scratch.alloc(hipk::running_median_wide_scratch_bytes(n_in)))) return rc;
  auto launch = [&]() {
    return wide ? hipk::launch_running_median_wide(din.p, n_in, W, dout.p, scratch.p, nullptr)
                : hipk::launch_running_median(din.p, n_in, W, dout.p, nullptr);
  };
  // pinned bounce buffer (no runtime pageable-copy path, see Impl::copy_out)
  PinnedBuf<float> hbuf;
  if ((rc = hbuf.alloc(std::max(in.size(), n_out)))) return rc;
  std::memcpy(hbuf.p, in.data(), in.size() * sizeof(float));
  BRP_HIP_CHECK(hipMemcpy(din.p, hbuf.p, in.size() * sizeof(float), hipMemcpyHostToDevice),
                RADPUL_HIP_MEM_COPY_HOST_DEVICE);
  hipEvent_t e0, e1;
  BRP_HIP_CHECK(hipEventCreate(&e0), RADPUL_HIP_DEVICE_SET);
  BRP_HIP_CHECK(hipEventCreate(&e1), RADPUL_HIP_DEVICE_SET);
  BRP_HIP_CHECK(launch(), RADPUL_HIP_KERNEL_INVOKE);
  BRP_HIP_CHECK(hipEventRecord(e0, nullptr), RADPUL_HIP_KERNEL_INVOKE);
  for (int r = 0; r < reps; ++r) BRP_HIP_CHECK(launch(), RADPUL_HIP_KERNEL_INVOKE);
  BRP_HIP_CHECK(hipEventRecord(e1, nullptr), RADPUL_HIP_KERNEL_INVOKE);
  BRP_HIP_CHECK(hipEventSynchronize(e1), RADPUL_HIP_KERNEL_INVOKE);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  if (ms_per_call) *ms_per_call = reps > 0 ? ms / reps : 0.0;
  out.resize(n_out);
  BRP_HIP_CHECK(hipMemcpy(hbuf.p, dout.p, n_out * sizeof(float), hipMemcpyDeviceToHost),
                RADPUL_HIP_MEM_COPY_DEVICE_HOST);
  std::memcpy(out.data(), hbuf.p, n_out * sizeof(float));
  return 0;
}

int HipEngine::init(int device, int batch) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    log_message(LOG_ERROR, true, "No HIP device available.\n");
    return RADPUL_HIP_DEVICE_FIND;
  }
  if (device < 0) {
    const char* env = std::getenv("BRP_DEVICE");
    device = env ? std::atoi(env) : best_device(ndev);
  }
  if (device >= ndev) {
    log_message(LOG_ERROR, true, "Requested device %d but only %d present.\n", device, ndev);
    return RADPUL_HIP_DEVICE_SET;
  }
  BRP_HIP_CHECK(hipSetDevice(device), RADPUL_HIP_DEVICE_SET);
  if (g_blocking_sync) {
    // host waits sleep instead of spinning (reference CU_CTX_BLOCKING_SYNC with
    // fallback to automatic scheduling, cuda/app/demod_binary_cuda.cu:126-137)
    if (hipSetDeviceFlags(hipDeviceScheduleBlockingSync) != hipSuccess) {
      (void)hipGetLastError();
      log_message(LOG_WARN, true, "Blocking synchronisation unavailable (context exists): automatic scheduling.\n");
    }
  }
  impl_->device = device;
  impl_->batch = batch > 0 ? batch : 4;
  {
    const char* e = std::getenv("BRP_SERIAL");
    const int sv = e ? std::atoi(e) : kDefaultSerial;
    impl_->serial = std::max(1, std::min(sv, static_cast<int>(hipk::kHsMaxBatch) / impl_->batch));
  }
  impl_->batch_req = impl_->batch;
  impl_->serial_req = impl_->serial;
  BRP_HIP_CHECK(hipStreamCreateWithFlags(&impl_->stream, hipStreamNonBlocking), RADPUL_HIP_DEVICE_SET);
  for (auto& o : impl_->io) {
    BRP_HIP_CHECK(hipEventCreate(&o.ev0), RADPUL_HIP_DEVICE_SET);
    BRP_HIP_CHECK(hipEventCreate(&o.ev1), RADPUL_HIP_DEVICE_SET);
  }
  BRP_HIP_CHECK(hipEventCreate(&impl_->ev_w0), RADPUL_HIP_DEVICE_SET);
  BRP_HIP_CHECK(hipEventCreate(&impl_->ev_w1), RADPUL_HIP_DEVICE_SET);
  BRP_HIP_CHECK(hipEventCreateWithFlags(&impl_->ev_adopt, hipEventDisableTiming), RADPUL_HIP_DEVICE_SET);
  impl_->select_io(0);
  hipDeviceProp_t prop;
  BRP_HIP_CHECK(hipGetDeviceProperties(&prop, device), RADPUL_HIP_DEVICE_PROP);
  log_message(LOG_INFO, true, "Using HIP device #%d: %s (%s, %d CUs, %.1f GB)\n", device, prop.name,
              prop.gcnArchName, prop.multiProcessorCount, prop.totalGlobalMem / 1e9);
  impl_->num_cus = static_cast<uint32_t>(prop.multiProcessorCount);
  impl_->arch = prop.gcnArchName;
  return 0;
}

namespace {
bool same_geometry(const SearchGeometry& a, const SearchGeometry& b) {
  return a.nsamples == b.nsamples && a.n_unpadded == b.n_unpadded && a.fft_size == b.fft_size &&
         a.window_2 == b.window_2 && a.fundamental_idx_hi == b.fundamental_idx_hi &&
         a.harmonic_idx_hi == b.harmonic_idx_hi && a.dt == b.dt && a.step_inv == b.step_inv;
}
}  // namespace

// One-time costs of the process's first work, paid here so that a caller can
// overlap them with other start-up (search.cpp: pipeline 0's warm-up runs
// while the other pipelines' streams are created): the device modules' code
// objects (loaded at the first launch otherwise, ~14 ms), the runtime's copy
// kernels (first copy on a stream, ~11 ms), the pinned stage.
int HipEngine::warm_up() {
  Impl& d = *impl_;
  trace::Range range("brp:warm_up");
  BRP_HIP_CHECK(hipSetDevice(d.device), RADPUL_HIP_DEVICE_SET);
  for (hipError_t (*f)() : {hipk::preload_fft_passes, hipk::preload_harmonic_sum, hipk::preload_whiten,
                            hipk::preload_resample, hipk::preload_bluestein, hipk::preload_rmed_wide})
    if (f() != hipSuccess) (void)hipGetLastError();  // only an optimisation: the launch loads it otherwise
  int rc;
  if ((rc = d.stage.reserve(Impl::kStageChunk))) return rc;
  // a small copy each way (the runtime's copy kernels) and a large one (its
  // DMA engine path: the first 2 MB series upload took ~8 ms more than later ones)
  DevBuf<uint8_t> probe;
  constexpr size_t kLarge = 4u << 20;
  if ((rc = probe.alloc(kLarge))) return rc;
  std::memset(d.stage.p, 0, kLarge);
  for (size_t n : {size_t{64}, kLarge}) {
    BRP_HIP_CHECK(copy_sync(probe.p, d.stage.p, n, hipMemcpyHostToDevice, d.stream), RADPUL_HIP_MEM_COPY_HOST_DEVICE);
    BRP_HIP_CHECK(copy_sync(d.stage.p, probe.p, n, hipMemcpyDeviceToHost, d.stream), RADPUL_HIP_MEM_COPY_DEVICE_HOST);
  }
  return 0;
}

int HipEngine::setup(const SearchGeometry& g, const std::vector<float>& series, float mu0) {
  if (series.size() < g.n_unpadded) return RADPUL_EVAL;
  return setup_impl(g, series.data(), nullptr, -1, mu0);
}

int HipEngine::setup_packed(const SearchGeometry& g, const WorkUnit& wu, float mu0) {
  if (wu.samples.size() < g.n_unpadded || wu.packed.empty()) return RADPUL_EVAL;
  return setup_impl(g, wu.samples.data(), nullptr, -1, mu0, &wu);
}

int HipEngine::setup_peer(const HipEngine& src) {
  const Impl& s = *src.impl_;
  if (!s.ready || s.slots != 1) return RADPUL_EVAL;
  // the source's whitening ran on its own stream
  BRP_HIP_CHECK(hipSetDevice(s.device), RADPUL_HIP_DEVICE_SET);
  BRP_HIP_CHECK(hipStreamSynchronize(s.stream), RADPUL_HIP_MEM_COPY_HOST_DEVICE);
  return setup_impl(s.g, nullptr, s.series_in(), s.device, s.mu0s[0]);
}

int HipEngine::upload_series0(const float* host, const float* dev_src, int src_device, const WorkUnit* packed) {
  Impl& d = *impl_;
  const size_t bytes = d.g.n_unpadded * sizeof(float);
  if (packed != nullptr) {
    // the payload (n/2 bytes for 4-bit: 2 MB instead of 16.8 MB on the
    // benchmark WU), unpacked on the device into slot 0
    trace::Range up("brp:series_upload_packed");
    const size_t nb = packed->packed.size();
    int rc;
    if (d.wu_packed.n < nb && (rc = d.wu_packed.alloc(nb))) return rc;
    BRP_HIP_CHECK(d.copy_in(d.wu_packed.p, packed->packed.data(), nb), RADPUL_HIP_MEM_COPY_HOST_DEVICE);
    BRP_HIP_CHECK(hipk::launch_unpack(d.wu_packed.p, static_cast<uint32_t>(nb), packed->four_bit, packed->header.scale,
                                      d.series.p, d.g.n_unpadded, d.stream),
                  RADPUL_HIP_KERNEL_INVOKE);
    return 0;  // stream-ordered before everything that reads the series (the WU payload outlives the copy)
  }
  if (dev_src != nullptr) {
    // device to device: same device, or a peer over xGMI (no host round trip)
    trace::Range up("brp:series_peer_copy");
    BRP_HIP_CHECK(hipMemcpyPeerAsync(d.series.p, d.device, dev_src, src_device, bytes, d.stream),
                  RADPUL_HIP_MEM_COPY_HOST_DEVICE);
    BRP_HIP_CHECK(hipStreamSynchronize(d.stream), RADPUL_HIP_MEM_COPY_HOST_DEVICE);
    d.st.peer_series_copies += 1;
    return 0;
  }
  trace::Range up("brp:series_upload");
  BRP_HIP_CHECK(d.copy_in(d.series.p, host, bytes), RADPUL_HIP_MEM_COPY_HOST_DEVICE);
  return 0;
}

int HipEngine::setup_impl(const SearchGeometry& g, const float* host_series, const float* dev_series, int src_device,
                          float mu0, const WorkUnit* packed) {
  trace::Range range("brp:engine_setup");
  Impl& d = *impl_;
  BRP_HIP_CHECK(hipSetDevice(d.device), RADPUL_HIP_DEVICE_SET);
  d.own_series();
  if (d.ready && same_geometry(d.g, g)) {
    // next work unit of the same shape (or the same WU again): buffers, tables
    // and captured graphs stay valid; only the series and its mean change
    d.g = g;
    d.mu0s.assign(d.slots, 0.0f);
    d.mu0s[0] = mu0;
    return upload_series0(host_series, dev_series, src_device, packed);
  }
  d.ready = false;
  for (auto& kv : d.graphs) (void)hipGraphExecDestroy(kv.second);
  d.graphs.clear();
  d.g = g;
  d.mu0s.assign(d.slots, 0.0f);
  d.mu0s[0] = mu0;
  d.bs = g.nsamples % 2 != 0 || !make_fft_plan(g.nsamples / 2, d.plan);
  d.bs_pair = false;
  d.batch = d.batch_req;
  d.serial = d.serial_req;
  if (d.bs) {
    // any other length (every padding -P the reference accepts): chirp-z
    // transform over the smallest factorable convolution length
    d.bs_Mb = (g.nsamples % 2) ? g.nsamples : g.nsamples / 2;
    d.bs_pair = (g.nsamples % 2) != 0 &&
                (std::getenv("BRP_BS_PAIR") == nullptr || std::atoi(std::getenv("BRP_BS_PAIR")) != 0);
    if (d.bs_pair && d.batch == 1) {  // launch groups of two templates: one transform each
      d.batch = 2;
      d.serial = std::max(1, d.serial / 2);
    }
    if (!make_bluestein_plan(d.bs_Mb, d.plan)) {
      log_message(LOG_ERROR, true, "No FFT plan for length %u.\n", g.nsamples);
      return RADPUL_HIP_FFT_PLAN;
    }
    d.bs_rev = hipk::chirp_rev_supported(d.plan) &&
               (std::getenv("BRP_BS_REV") == nullptr || std::atoi(std::getenv("BRP_BS_REV")) != 0);
    log_message(LOG_INFO, true, "FFT length %u: chirp-z transform of length %u over %u = %u x %u x %u points%s.\n",
                g.nsamples, d.bs_Mb, d.plan.M, d.plan.L1, d.plan.L2, d.plan.L3, d.bs_rev ? " (transposed)" : "");
  }
  // measured settings for this (arch, M) from the plan wisdom; environment wins
  const PlanWisdom wis = load_wisdom(wisdom_path(), d.arch, d.plan.M);
  if (wis.found)
    log_message(LOG_DEBUG, true, "Plan wisdom for %s M=%u: persist %d\n", d.arch.c_str(), d.plan.M,
                wis.persist_per_cu);
  if (wis.persist_per_cu >= 0) d.persist_per_cu = static_cast<uint32_t>(wis.persist_per_cu);
  if (const char* e = std::getenv("BRP_PERSIST")) d.persist_per_cu = static_cast<uint32_t>(std::atoi(e));
  d.plan.persist_wgs = d.persist_per_cu * d.num_cus;
  log_message(LOG_DEBUG, true, "FFT plan: N=%u M=%u = %u x %u x %u\n", g.nsamples, d.plan.M, d.plan.L1, d.plan.L2,
              d.plan.L3);
  const uint32_t limit = std::min(g.harmonic_idx_hi, g.fft_size);
  d.ps_stride = std::max<uint32_t>((std::max(limit, g.fundamental_idx_hi) + 63) / 64 * 64, 64);
  // first harmonic-sum tile: i_start == 8 mod 16 and <= window_2 (-8 below 8)
  d.i_start = (g.window_2 >= 8) ? static_cast<int32_t>(((g.window_2 - 8) / 16) * 16 + 8) : -8;
  // candidate keys sized to the geometry: bins < 2^bin_bits, and at most the
  // templates per submitted batch the remaining key bits address
  d.bin_bits = hipk::hs_bin_bits(std::max<uint32_t>(g.fundamental_idx_hi, 2));
  const uint32_t key_templates = hipk::hs_key_templates(d.bin_bits);
  if (key_templates == 0) {
    log_message(LOG_ERROR, true, "fundamental_idx_hi %u: more bins than a candidate key addresses (2^%u).\n",
                g.fundamental_idx_hi, hipk::kHsMaxBinBits);
    return RADPUL_EVAL;
  }
  while (static_cast<uint32_t>(d.slot_cap()) > key_templates) {
    if (d.serial > 1) d.serial = std::max(1, static_cast<int>(key_templates) / d.batch);
    else d.batch = static_cast<int>(key_templates);
  }
  d.dense_stride = std::max<uint32_t>((g.fundamental_idx_hi + 63) / 64 * 64, 64);
  if (const char* e = std::getenv("BRP_HS_CAP")) {
    // fault injection (small lists overflow early); never below what the
    // bounded output of a full batch emits (100 per template and level, +28 % for ties)
    // (BRP_FAULT=hs_cap_raw: taken as is, so that the bounded output itself
    // overflows -- the tie-storm path of complete())
    const uint32_t min_cap =
        fault_enabled("hs_cap_raw") ? 1u : static_cast<uint32_t>(d.slot_cap()) * kNumHarmonicLevels * 128u;
    d.cap = std::max<uint32_t>(min_cap, static_cast<uint32_t>(std::atol(e)));
    d.kcopy = std::min(d.kcopy, d.cap);
    d.inplace_max = std::min(d.inplace_max, d.kcopy);
  }
  d.select_forced = std::getenv("BRP_HS_SELECT") != nullptr && std::atoi(std::getenv("BRP_HS_SELECT")) != 0;
  d.select_mode = d.select_forced;
  d.sel_dense.release();
  int rc;
  if (d.select_mode && (rc = d.ensure_select())) return rc;
  const size_t B = static_cast<size_t>(d.batch);
  if ((rc = d.series.alloc(static_cast<size_t>(d.slots) * g.n_unpadded))) return rc;
  if ((rc = d.buf.alloc(B * d.plan.M))) return rc;
  if ((rc = d.ps.alloc(B * d.ps_stride))) return rc;
  d.hs_prune = std::getenv("BRP_HS_FULL") == nullptr || std::atoi(std::getenv("BRP_HS_FULL")) == 0;
  d.hs_cell_shift = (std::getenv("BRP_HS_CELL") && std::atoi(std::getenv("BRP_HS_CELL")) == 4) ? 2 : 3;
  if (const char* e = std::getenv("BRP_FG_INPLACE_MAX"))
    d.inplace_max = std::min<uint32_t>(d.kcopy, static_cast<uint32_t>(std::max(0, std::atoi(e))));
  d.hs_direct = std::getenv("BRP_HS_DIRECT") == nullptr || std::atoi(std::getenv("BRP_HS_DIRECT")) != 0;
  d.p3_cells = std::getenv("BRP_P3_CELLS") != nullptr && std::atoi(std::getenv("BRP_P3_CELLS")) != 0;
  d.hs_cells_cpt = (std::getenv("BRP_HS_CELLS_CPT") && std::atoi(std::getenv("BRP_HS_CELLS_CPT")) == 4) ? 4u : 1u;
  d.hs_xcd = std::getenv("BRP_HS_XCD") != nullptr && std::atoi(std::getenv("BRP_HS_XCD")) == 1;
  d.lds_pass1 = std::getenv("BRP_P1_LDS") != nullptr && std::atoi(std::getenv("BRP_P1_LDS")) == 1;
  d.mid_waves = std::getenv("BRP_MID_WAVES") != nullptr && std::atoi(std::getenv("BRP_MID_WAVES")) == 1;
  if ((rc = d.pyr.alloc(B * hipk::hs_pyr_stride(d.ps_stride)))) return rc;
  if ((rc = d.partials.alloc(B * d.plan.wg1()))) return rc;  // pass-1 partial sums (P1_RESAMPLE / P1_CHIRP*)
  if (d.bs) {
    if ((rc = d.bs_a.alloc(B * d.plan.M)) || (rc = d.bs_h.alloc(d.plan.M))) return rc;
    if (d.bs_rev && (rc = d.bs_hp.alloc(d.plan.M))) return rc;
    const auto& ch = twiddles_cached(2ull * d.bs_Mb);
    if ((rc = d.upload(d.bs_chirp_hi, ch.first)) || (rc = d.upload(d.bs_chirp_lo, ch.second))) return rc;
  } else {
    d.bs_a.release();
    d.bs_h.release();
  }
  if (!d.bs || !d.bs_rev) d.bs_hp.release();
  if ((rc = d.delta.alloc(B))) return rc;
  const size_t BS = static_cast<size_t>(d.slot_cap());  // templates per I/O slot
  d.thr_bytes = (BS * hipk::kHsThrStride * sizeof(float) + 63) / 64 * 64;
  const size_t in_bytes = d.thr_bytes + sizeof(TemplateDev) * BS;
  {
    const char* fg = std::getenv("BRP_FG");
    const std::string f = fg ? fg : "";
    // measured (profiles/README.md): parameters in place +1.9 %; results in
    // place +1.0-1.6 % once the harmonic sum no longer held LDS (round 3, 5
    // interleaved rounds); default "both"
    d.fg_in = f.empty() || f == "in" || f == "both" || f == "1";
    d.fg_out = f.empty() || f == "out" || f == "both" || f == "1";
  }
  for (int i = 0; i < Impl::kIoSlots; ++i) {
    Impl::BatchIO& o = d.io[i];
    o.pending = false;
    if ((rc = o.in.alloc(in_bytes, d.fg_in))) return rc;
    uint8_t* in_host =
        d.fg_in ? static_cast<uint8_t*>(host_view(d.device, o.in.p, in_bytes, d.stream, d.stage)) : nullptr;
    if (d.fg_in && in_host == nullptr) {
      log_message(LOG_WARN, true, "Fine-grained device memory is not host visible; copying the batch parameters.\n");
      d.fg_in = false;
      if ((rc = o.in.alloc(in_bytes))) return rc;
      if (i > 0) return RADPUL_EMEM;  // slot 0 was host visible: inconsistent
    }
    if ((rc = o.cands.alloc(1 + d.cap, d.fg_out))) return rc;
    if (d.fg_in) {
      o.h_in_p = in_host;
    } else {
      if ((rc = o.h_in.alloc(in_bytes))) return rc;
      o.h_in_p = o.h_in.p;
    }
    uint2* cands_host =
        d.fg_out ? static_cast<uint2*>(host_view(d.device, o.cands.p, sizeof(uint2) * (1 + d.kcopy), d.stream, d.stage))
                 : nullptr;
    if (d.fg_out && cands_host == nullptr) {
      log_message(LOG_WARN, true, "Fine-grained device memory is not host visible; copying the results.\n");
      d.fg_out = false;
      if ((rc = o.cands.alloc(1 + d.cap))) return rc;
      if (i > 0) return RADPUL_EMEM;
    }
    if (d.fg_out) {
      o.h_cands_p = cands_host;  // non-owning view
    } else {
      if ((rc = o.h_cands.alloc(1 + d.kcopy))) return rc;
      o.h_cands_p = o.h_cands.p;
    }
  }
  d.io_next = d.io_head = 0;
  d.select_io(0);
  const auto& twc = twiddles_cached(2ull * g.nsamples);
  const std::vector<float2>& hi = twc.first;
  const std::vector<float2>& lo = twc.second;
  if ((rc = d.tw_hi.alloc(hi.size()))) return rc;
  if ((rc = d.tw_lo.alloc(lo.size()))) return rc;
  BRP_HIP_CHECK(d.copy_in(d.tw_hi.p, hi.data(), hi.size() * sizeof(float2)), RADPUL_HIP_MEM_COPY_HOST_DEVICE);
  BRP_HIP_CHECK(d.copy_in(d.tw_lo.p, lo.data(), lo.size() * sizeof(float2)), RADPUL_HIP_MEM_COPY_HOST_DEVICE);
  if ((rc = d.build_tables())) return rc;
  if (d.bs) {
    BRP_HIP_CHECK(d.bs_make_h(), RADPUL_HIP_KERNEL_INVOKE);
    if (d.bs_rev)
      BRP_HIP_CHECK(hipk::launch_bs_rows(d.bs_h.p, d.bs_hp.p, d.plan.L1, d.plan.L2, d.plan.L3, d.stream),
                    RADPUL_HIP_KERNEL_INVOKE);
    BRP_HIP_CHECK(hipStreamSynchronize(d.stream), RADPUL_HIP_KERNEL_INVOKE);
  }
  if ((rc = upload_series0(host_series, dev_series, src_device, packed))) return rc;
  log_mem_status(d.device, "after setup");
  d.ready = true;
  return 0;
}

int HipEngine::upload_series(const std::vector<float>& series, float mu0) { return load_slot(0, series, mu0); }

int HipEngine::adopt_series(const HipEngine& src) {
  Impl& d = *impl_;
  const Impl& s = *src.impl_;
  // any number of work-unit slots (multi-WU batching), the same on both sides
  if (!d.ready || !s.ready || d.device != s.device || d.slots != s.slots || !same_geometry(d.g, s.g))
    return RADPUL_EVAL;
  trace::Range range("brp:adopt_series");
  BRP_HIP_CHECK(hipSetDevice(d.device), RADPUL_HIP_DEVICE_SET);
  d.g = s.g;
  d.mu0s = s.mu0s;
  static const bool share = std::getenv("BRP_SHARE_SERIES") == nullptr || std::atoi(std::getenv("BRP_SHARE_SERIES")) != 0;
  // everything queued on the source's stream so far (upload, whitening) comes
  // before this pipeline's next work: a device-side dependency, no host wait
  BRP_HIP_CHECK(hipEventRecord(d.ev_adopt, s.stream), RADPUL_HIP_MEM_COPY_HOST_DEVICE);
  BRP_HIP_CHECK(hipStreamWaitEvent(d.stream, d.ev_adopt, 0), RADPUL_HIP_MEM_COPY_HOST_DEVICE);
  const float* want = share ? s.series_in() : nullptr;
  if (want != d.shared_series) {
    d.shared_series = want;
    for (auto& kv : d.graphs) (void)hipGraphExecDestroy(kv.second);  // captured series pointer changed
    d.graphs.clear();
  }
  if (want != nullptr) {
    // the source may itself read a third engine's series: follow that token
    d.adopted_token = s.shared_series != nullptr ? s.adopted_token : s.series_token;
    d.adopted_gen = s.shared_series != nullptr ? s.adopted_gen : s.series_token->load();
  } else {
    d.adopted_token.reset();
  }
  if (!share)
    BRP_HIP_CHECK(copy_sync(d.series.p, s.series_in(), static_cast<size_t>(d.slots) * d.g.n_unpadded * sizeof(float),
                            hipMemcpyDeviceToDevice, d.stream),
                  RADPUL_HIP_MEM_COPY_HOST_DEVICE);
  return 0;
}

int HipEngine::set_slots(uint32_t k) {
  Impl& d = *impl_;
  if (k == 0 || k > (1u << 16)) return RADPUL_EVAL;
  if (k != d.slots) {
    d.slots = k;
    d.ready = false;  // the next setup() reallocates the series buffer
    d.bump_series();
  }
  return 0;
}

uint32_t HipEngine::slots() const { return impl_->slots; }

bool HipEngine::ps_fp16() const { return impl_->ps_fp16; }

void HipEngine::set_ps_fp16(bool on) {
  Impl& d = *impl_;
  if (on == d.ps_fp16) return;
  d.ps_fp16 = on;
  for (auto& kv : d.graphs) (void)hipGraphExecDestroy(kv.second);  // captured arguments changed
  d.graphs.clear();
}

int HipEngine::load_slot(uint32_t k, const std::vector<float>& series, float mu0) {
  Impl& d = *impl_;
  if (!d.ready || k >= d.slots || series.size() < d.g.n_unpadded) return RADPUL_EVAL;
  BRP_HIP_CHECK(hipSetDevice(d.device), RADPUL_HIP_DEVICE_SET);
  d.own_series();
  d.mu0s[k] = mu0;
  BRP_HIP_CHECK(d.copy_in(d.series.p + static_cast<size_t>(k) * d.g.n_unpadded, series.data(),
                          d.g.n_unpadded * sizeof(float)),
                RADPUL_HIP_MEM_COPY_HOST_DEVICE);
  return 0;
}

bool HipEngine::prepared_for(const SearchGeometry& g) const {
  return impl_->ready && impl_->slots == 1 && same_geometry(impl_->g, g);
}

bool HipEngine::ready_for(const SearchGeometry& g) const { return impl_->ready && same_geometry(impl_->g, g); }

int HipEngine::whiten(const SearchOptions& opt, const std::vector<ZapRange>& zaps, std::vector<float>& series,
                      uint32_t slot, bool copy_back) {
  Impl& d = *impl_;
  trace::Range range("brp:whiten");
  if (slot >= d.slots) return RADPUL_EVAL;
  d.own_series();
  float* slot_series = d.series.p + static_cast<size_t>(slot) * d.g.n_unpadded;
  const SearchGeometry& g = d.g;
  d.settle_whiten(true);  // the previous whitening's host noise arrays are free again
  auto t0 = std::chrono::steady_clock::now();
  BRP_HIP_CHECK(hipEventRecord(d.ev_w0, d.stream), RADPUL_HIP_KERNEL_INVOKE);
  int32_t seed;
  std::memcpy(&seed, series.data(), sizeof(seed));
  log_message(LOG_INFO, true, "Seed for random number generator is %d.\n", seed);
  const uint32_t fft_size = g.fft_size, M = d.plan.M;
  if (fft_size < opt.window) return RADPUL_EVAL;
  DevBuf<float2>& spec = d.w_spec;
  DevBuf<float>& psw = d.w_psw;
  DevBuf<float>& med = d.w_med;
  int rc;
  const uint32_t white_size = fft_size - opt.window + 1;
  // scratch kept across work units of the same shape
  if (spec.n < fft_size && (rc = spec.alloc(fft_size))) return rc;
  if (psw.n < fft_size && (rc = psw.alloc(fft_size))) return rc;
  if (med.n < white_size && (rc = med.alloc(white_size))) return rc;
  float2* work = d.buf.p;  // M complex scratch (batch slot 0)
  const hipk::TwiddleTable tw = d.twt();
  hipStream_t s = d.stream;
  const bool odd = (g.nsamples & 1u) != 0;
  // forward r2c of the zero-padded series
  if (d.bs) {
    hipk::BsInArgs ab = d.bs_in();
    ab.real_in = slot_series;
    ab.n_real = g.n_unpadded;
    BRP_HIP_CHECK(hipk::launch_bs_chirp_in(odd ? hipk::BS_IN_REAL1 : hipk::BS_IN_REAL2, ab, 1, nullptr, s),
                  RADPUL_HIP_KERNEL_INVOKE);
    BRP_HIP_CHECK(d.bs_convolve(1), RADPUL_HIP_KERNEL_INVOKE);
    BRP_HIP_CHECK(hipk::launch_bs_spec(d.bs_a.p, d.bs_Mb, g.nsamples, tw, fft_size, spec.p, s),
                  RADPUL_HIP_KERNEL_INVOKE);
  } else {
  hipk::Pass1Args a1{};
  a1.out = work;
  a1.L2L3 = d.plan.L2 * d.plan.L3;
  a1.L3 = d.plan.L3;
  a1.tw = tw;
  a1.tb = d.tables();
  a1.real_in = slot_series;
  a1.n_real = g.n_unpadded;
  BRP_HIP_CHECK(hipk::launch_pass1(d.plan, hipk::P1_REAL, a1, 1, s), RADPUL_HIP_KERNEL_INVOKE);
  hipk::Pass2Args a2{};
  a2.buf = work;
  a2.L1 = d.plan.L1;
  a2.L2L3 = d.plan.L2 * d.plan.L3;
  a2.L3 = d.plan.L3;
  a2.tw = tw;
  a2.tb = d.tables();
  BRP_HIP_CHECK(hipk::launch_pass2(d.plan, a2, 1, s), RADPUL_HIP_KERNEL_INVOKE);
  hipk::Pass3Args a3{};
  a3.buf = work;
  a3.L1 = d.plan.L1;
  a3.L2 = d.plan.L2;
  a3.L3 = d.plan.L3;
  a3.C = d.plan.L1 * d.plan.L2;
  a3.M = M;
  a3.tw = tw;
  a3.tb = d.tables();
  a3.limit = fft_size;
  a3.spec = spec.p;
  BRP_HIP_CHECK(hipk::launch_pass3(d.plan, hipk::P3_COMPLEX, a3, 1, s), RADPUL_HIP_KERNEL_INVOKE);
  }
  BRP_HIP_CHECK(hipk::launch_whiten_power(spec.p, fft_size, psw.p, s), RADPUL_HIP_KERNEL_INVOKE);
  hipError_t rme = hipErrorInvalidConfiguration;
  if (hipk::running_median_supported(opt.window)) rme = hipk::launch_running_median(psw.p, fft_size, opt.window, med.p, s);
  if (rme != hipErrorInvalidConfiguration) {
    BRP_HIP_CHECK(rme, RADPUL_HIP_KERNEL_INVOKE);
  } else {
    // wide windows (up to the reference's 250 000): device radix sort + median walk
    const size_t bytes = hipk::running_median_wide_scratch_bytes(fft_size);
    if (d.w_rmed.n < bytes && (rc = d.w_rmed.alloc(bytes))) return rc;
    BRP_HIP_CHECK(hipk::launch_running_median_wide(psw.p, fft_size, opt.window, med.p, d.w_rmed.p, s),
                  RADPUL_HIP_KERNEL_INVOKE);
  }
  BRP_HIP_CHECK(hipk::launch_whiten_scale(spec.p, med.p, white_size, g.window_2, s), RADPUL_HIP_KERNEL_INVOKE);
  // RFI zapping: noise drawn on the host in the reference order (GSL-compatible RNG)
  ZapNoise noise;
  trace::range_push("brp:zap_noise");
  make_zap_noise(seed, g, opt, zaps, noise);
  DevBuf<uint32_t>& zbins = d.w_zbins;
  DevBuf<float2>& znoise = d.w_znoise;
  const uint32_t nz = static_cast<uint32_t>(noise.bin.size());
  // host sources of the async copies must outlive them: engine members,
  // reused only once this whitening's end event has passed (settle_whiten)
  std::vector<float2> zn;
  std::vector<uint32_t> zb;
  if (nz) {
    // overlapping zap ranges hit a bin more than once: sequentially the last
    // draw wins, so keep only that one (the device writes bins in parallel)
    std::unordered_map<uint32_t, uint32_t> last;
    last.reserve(nz);
    for (uint32_t i = 0; i < nz; ++i) last[noise.bin[i]] = i;
    for (uint32_t i = 0; i < nz; ++i) {
      if (last[noise.bin[i]] != i) continue;
      zb.push_back(noise.bin[i]);
      zn.push_back(make_float2(noise.re[i], noise.im[i]));
    }
  }
  const uint32_t nzu = static_cast<uint32_t>(zb.size());
  trace::range_pop();
  if (nzu) {
    // kept across passes (a hipFree per pass would synchronise the device)
    if (zbins.n < nzu && (rc = zbins.alloc(nzu))) return rc;
    if (znoise.n < nzu && (rc = znoise.alloc(nzu))) return rc;
    if ((rc = d.w_zb_host.reserve(nzu)) || (rc = d.w_zn_host.reserve(nzu))) return rc;
    std::memcpy(d.w_zb_host.p, zb.data(), nzu * sizeof(uint32_t));
    std::memcpy(d.w_zn_host.p, zn.data(), nzu * sizeof(float2));
    BRP_HIP_CHECK(memcpy_async(zbins.p, d.w_zb_host.p, nzu * sizeof(uint32_t), hipMemcpyHostToDevice, s),
                  RADPUL_HIP_MEM_COPY_HOST_DEVICE);
    BRP_HIP_CHECK(memcpy_async(znoise.p, d.w_zn_host.p, nzu * sizeof(float2), hipMemcpyHostToDevice, s),
                  RADPUL_HIP_MEM_COPY_HOST_DEVICE);
    BRP_HIP_CHECK(hipk::launch_zap(spec.p, fft_size, zbins.p, znoise.p, nzu, s), RADPUL_HIP_KERNEL_INVOKE);
  }
  // inverse c2r: tangle, conj-FFT, natural order, scale by 1/sqrt(N), keep n_unpadded
  const float inv_scale = static_cast<float>(1.0 / std::sqrt(static_cast<float>(g.nsamples)));
  DevBuf<float2>& z = d.w_z;
  const uint32_t Mz = d.bs ? d.bs_Mb : M;  // packed half length (even N)
  if (!odd && z.n < Mz && (rc = z.alloc(Mz))) return rc;
  if (!odd)
    BRP_HIP_CHECK(hipk::launch_tangle(spec.p, Mz, fft_size, g.window_2, tw, z.p, s), RADPUL_HIP_KERNEL_INVOKE);
  if (d.bs) {
    hipk::BsInArgs ab = d.bs_in();
    ab.cplx_in = odd ? spec.p : z.p;
    ab.w2 = g.window_2;
    ab.fft_size = fft_size;
    BRP_HIP_CHECK(hipk::launch_bs_chirp_in(odd ? hipk::BS_IN_HERM_CONJ : hipk::BS_IN_CONJ, ab, 1, nullptr, s),
                  RADPUL_HIP_KERNEL_INVOKE);
    BRP_HIP_CHECK(d.bs_convolve(1), RADPUL_HIP_KERNEL_INVOKE);
    BRP_HIP_CHECK(hipk::launch_bs_real_out(d.bs_a.p, d.bs_Mb, g.nsamples, inv_scale, slot_series, g.n_unpadded, s),
                  RADPUL_HIP_KERNEL_INVOKE);
  } else {
    hipk::Pass1Args a1{};
    a1.out = work;
    a1.L2L3 = d.plan.L2 * d.plan.L3;
    a1.L3 = d.plan.L3;
    a1.tw = tw;
    a1.tb = d.tables();
    a1.cplx_in = z.p;
    BRP_HIP_CHECK(hipk::launch_pass1(d.plan, hipk::P1_COMPLEX_CONJ, a1, 1, s), RADPUL_HIP_KERNEL_INVOKE);
    hipk::Pass2Args a2{};
    a2.buf = work;
    a2.L1 = d.plan.L1;
    a2.L2L3 = d.plan.L2 * d.plan.L3;
    a2.L3 = d.plan.L3;
    a2.tw = tw;
    a2.tb = d.tables();
    BRP_HIP_CHECK(hipk::launch_pass2(d.plan, a2, 1, s), RADPUL_HIP_KERNEL_INVOKE);
    hipk::Pass3PlainArgs ap{};
    ap.buf = work;
    ap.L1 = d.plan.L1;
    ap.L2 = d.plan.L2;
    ap.L3 = d.plan.L3;
    ap.C = d.plan.L1 * d.plan.L2;
    ap.tw = tw;
    ap.tb = d.tables();
    ap.scale = inv_scale;
    ap.real_out = slot_series;
    ap.n_out = g.n_unpadded;
    BRP_HIP_CHECK(hipk::launch_pass3_plain(d.plan, ap, s), RADPUL_HIP_KERNEL_INVOKE);
  }
  d.mu0s[slot] = 0.0f;  // whitened series has its DC (and first window_2 bins) removed
  if (copy_back) {
    {
      trace::Range wait("brp:whiten_wait");
      BRP_HIP_CHECK(hipStreamSynchronize(s), RADPUL_HIP_KERNEL_INVOKE);
    }
    BRP_HIP_CHECK(d.copy_out(series.data(), slot_series, g.n_unpadded * sizeof(float)), RADPUL_HIP_MEM_COPY_DEVICE_HOST);
    d.st.whiten_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return 0;
  }
  // the series stays on the device: the templates (this stream, or streams
  // ordered after it by adopt_series) run after the whitening without a host wait
  BRP_HIP_CHECK(hipEventRecord(d.ev_w1, s), RADPUL_HIP_KERNEL_INVOKE);
  d.w_pending = true;
  return 0;
}

int HipEngine::process(const TemplateInput* t, int n, const float thr[kNumHarmonicLevels],
                       std::vector<TemplateCands>& out) {
  return process(t, n, thr, 0, out);
}

int HipEngine::process(const TemplateInput* t, int n, const float* thr, int thr_stride,
                       std::vector<TemplateCands>& out) {
  Impl& d = *impl_;
  if (d.io_busy()) return RADPUL_EMISC;  // submitted batches must be completed first
  out.clear();
  out.resize(n);
  std::vector<TemplateCands> part;
  for (int off = 0; off < n; off += d.slot_cap()) {
    const int nb = std::min(d.slot_cap(), n - off);
    int rc = submit(t + off, nb, thr + static_cast<size_t>(off) * thr_stride, thr_stride);
    if (rc == 0) rc = complete(part);
    if (rc) return rc;
    for (int k = 0; k < nb; ++k) out[off + k] = std::move(part[k]);
  }
  return 0;
}

// two batches in flight per pipeline (BRP_INFLIGHT=1: one, the previous behaviour; 3: three)
int HipEngine::max_in_flight() const {
  static const int depth = std::getenv("BRP_INFLIGHT") ? std::max(1, std::atoi(std::getenv("BRP_INFLIGHT"))) : 2;
  return std::min(depth, Impl::kIoSlots);
}

int HipEngine::submit(const TemplateInput* t, int nb, const float* thr, int thr_stride) {
  Impl& d = *impl_;
  if (!d.ready || nb < 1 || nb > d.slot_cap()) return RADPUL_EMISC;
  if (!d.shared_series_valid()) {
    log_message(LOG_ERROR, true, "Pipeline reads a whitened series that was rewritten or freed since it was adopted.\n");
    return RADPUL_EVAL;
  }
  const int slot = d.io_next;
  if (d.io[slot].pending) return RADPUL_EMISC;  // more than kIoSlots batches in flight
  BRP_HIP_CHECK(hipSetDevice(d.device), RADPUL_HIP_DEVICE_SET);  // worker threads drive their own device
  const SearchGeometry& g = d.g;
  trace::Range launch("brp:batch_launch");
  d.select_io(slot);
  for (int k = 0; k < nb; ++k) {
    TemplateDev td{};
    td.p = make_resamp_params(g.nsamples, g.n_unpadded, g.fft_size, g.dt, g.step_inv, t[k].P, t[k].tau, t[k].Psi0);
    td.n_steps = resamp_n_steps(td.p, kSinLut, kCosLut);
    if (t[k].wu >= d.slots) return RADPUL_EVAL;
    td.wu = t[k].wu;
    td.mu0 = d.mu0s[td.wu];
    d.h_tmpl.p[k] = td;
    const float* th = thr + static_cast<size_t>(k) * thr_stride;
    for (int h = 0; h < kNumHarmonicLevels; ++h) d.h_thr.p[k * hipk::kHsThrStride + h] = th[h];
  }
  hipGraphExec_t exec = nullptr;
  // captured graphs differ by batch size, I/O slot and output path (compacting
  // or bounded select): entering or leaving select mode picks the other graph
  // instead of replaying one of the wrong path
  const int key = (nb * Impl::kIoSlots + slot) * 2 + (d.select_mode ? 1 : 0);
  auto it = d.graphs.find(key);
  // Direct launches into the stream by default: with two batches in flight the
  // launch cost is hidden, and replaying the batch as a HIP graph measured
  // 2-4 % slower (profiles/README.md). BRP_GRAPH=1 replays captured graphs.
  static const bool use_graph = std::getenv("BRP_GRAPH") != nullptr && std::atoi(std::getenv("BRP_GRAPH")) != 0;
  if (use_graph) {
    if (it == d.graphs.end()) {
      hipGraph_t graph;
      BRP_HIP_CHECK(hipStreamBeginCapture(d.stream, hipStreamCaptureModeThreadLocal), RADPUL_HIP_GRAPH);
      hipError_t e = d.enqueue(nb);
      hipError_t e2 = hipStreamEndCapture(d.stream, &graph);
      if (e != hipSuccess || e2 != hipSuccess) {
        log_message(LOG_ERROR, true, "Graph capture failed: %s / %s\n", hipGetErrorName(e), hipGetErrorName(e2));
        return RADPUL_HIP_GRAPH;
      }
      BRP_HIP_CHECK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0), RADPUL_HIP_GRAPH);
      (void)hipGraphDestroy(graph);
      d.graphs[key] = exec;
    } else {
      exec = it->second;
    }
  }
  if (d.fg_in) std::atomic_thread_fence(std::memory_order_seq_cst);  // BAR writes before the launch
  // One event per batch, at its end: every event record leaves the stream idle
  // for ~7 us (a start event cost 2-3 % of the bench, profiles/README.md round 3)
  if (use_graph) {
    BRP_HIP_CHECK(hipGraphLaunch(exec, d.stream), RADPUL_HIP_GRAPH);
  } else {
    BRP_HIP_CHECK(d.enqueue(nb), RADPUL_HIP_KERNEL_INVOKE);
  }
  BRP_HIP_CHECK(hipEventRecord(d.ev1, d.stream), RADPUL_HIP_KERNEL_INVOKE);
  d.io[slot].nb = nb;
  d.io[slot].pending = true;
  d.io[slot].sel = d.select_mode;
  d.io_next = (slot + 1) % Impl::kIoSlots;
  return 0;
}

int HipEngine::complete(std::vector<TemplateCands>& out) {
  Impl& d = *impl_;
  const int slot = d.io_head;
  Impl::BatchIO& o = d.io[slot];
  if (!o.pending) return RADPUL_EMISC;
  BRP_HIP_CHECK(hipSetDevice(d.device), RADPUL_HIP_DEVICE_SET);
  {
    trace::Range wait("brp:batch_wait");
    BRP_HIP_CHECK(hipEventSynchronize(o.ev1), RADPUL_HIP_KERNEL_INVOKE);
  }
  o.pending = false;
  d.io_head = (slot + 1) % Impl::kIoSlots;
  trace::Range decode("brp:batch_decode");
  const int nb = o.nb;
  // device time: from the end of the previous batch on this stream (its event
  // is not re-recorded before this completion unless every slot is in flight)
  float ms = 0;
  if (d.prev_done != nullptr && max_in_flight() < Impl::kIoSlots) (void)hipEventElapsedTime(&ms, d.prev_done, o.ev1);
  d.prev_done = d.io_busy() ? o.ev1 : nullptr;  // an idle stream restarts the chain
  d.st.busy_span_ms += ms;
  d.st.batches += 1;
  if (d.shared_series != nullptr) d.st.shared_series_batches += 1;
  d.st.templates += nb;
  uint32_t cnt = o.h_cands_p[0].x;
  bool ran_select = o.sel;
  if (cnt > d.cap && !o.sel) {
    // More above-threshold values than list slots (e.g. no -W: raw powers
    // exceed the chi^2 thresholds almost everywhere). Re-run this batch with
    // the bounded output (its parameters are still in the slot; the stream
    // orders the re-run after any batch queued behind this one) and keep that
    // mode for the following batches.
    log_message(LOG_DEBUG, true, "Candidate list overflow (%u > %u slots, %d templates): bounded output.\n", cnt,
                d.cap, nb);
    int rc;
    if ((rc = d.ensure_select())) return rc;
    // graphs are keyed by the output path, so none is destroyed here (the next
    // batch's graph launch may still be queued on the stream)
    d.select_mode = true;
    d.select_io(slot);
    if (d.fg_in) std::atomic_thread_fence(std::memory_order_seq_cst);
    BRP_HIP_CHECK(d.enqueue(nb), RADPUL_HIP_KERNEL_INVOKE);
    BRP_HIP_CHECK(hipEventRecord(o.ev1, d.stream), RADPUL_HIP_KERNEL_INVOKE);
    BRP_HIP_CHECK(hipEventSynchronize(o.ev1), RADPUL_HIP_KERNEL_INVOKE);
    d.st.overflow_reruns += 1;
    ran_select = true;
    cnt = o.h_cands_p[0].x;
    d.prev_done = nullptr;  // the statistics chain restarts
  }
  bool extra = false;  // the list was copied into list_host
  const uint2* src = o.h_cands_p + 1;
  if (cnt > d.cap) {
    // The bounded output itself overflowed: more values >= some template's
    // 100th-largest than list slots, i.e. a storm of exact ties at a 100th
    // place (the reference keeps inserting them one by one,
    // demod_binary.c:1310-1397). The bounded output is deterministic and its
    // counter kept counting past the cap, so one more run of the batch into a
    // list of exactly `cnt` slots emits every value: no input the reference
    // accepts ends in RADPUL_HIP_CAND_OVERFLOW.
    log_message(LOG_DEBUG, true, "Bounded output overflow (%u > %u slots, %d templates): list of %u slots.\n", cnt,
                d.cap, nb, cnt);
    // Every (template, level, bin) is emitted at most once, so a count above
    // nb x levels x fundamental bins is corrupt. The 32-bit counter cannot wrap
    // before that: the candidate key holds template << (bin_bits + 3), so
    // slot_cap x 8 x 2^bin_bits <= 2^32 (hs_key_templates).
    const uint64_t max_vals = static_cast<uint64_t>(nb) * kNumHarmonicLevels * std::max<uint32_t>(d.g.fundamental_idx_hi, 1);
    if (cnt > max_vals) {
      log_message(LOG_ERROR, true, "Bounded output counted %u values, more than the %llu a batch can emit.\n", cnt,
                  static_cast<unsigned long long>(max_vals));
      return RADPUL_HIP_CAND_OVERFLOW;
    }
    DevBuf<uint2> big;
    int rc;
    if ((rc = big.alloc(1 + static_cast<size_t>(cnt)))) return rc;
    const uint32_t cap0 = d.cap;
    const bool sel0 = d.select_mode;
    int rc2;
    if ((rc2 = d.ensure_select())) return rc2;
    d.select_io(slot);
    d.cands.p = big.p;  // the list of this run only (the slot's own list is untouched)
    d.cap = cnt;
    d.select_mode = true;
    hipError_t e = d.enqueue(nb);
    d.cap = cap0;
    d.select_mode = sel0;
    d.select_io(slot);
    BRP_HIP_CHECK(e, RADPUL_HIP_KERNEL_INVOKE);
    if ((rc = d.list_host.reserve(1 + static_cast<size_t>(cnt)))) return rc;
    BRP_HIP_CHECK(memcpy_async(d.list_host.p, big.p, (1 + static_cast<size_t>(cnt)) * sizeof(uint2), hipMemcpyDeviceToHost,
                                 d.stream),
                  RADPUL_HIP_MEM_COPY_DEVICE_HOST);
    BRP_HIP_CHECK(hipStreamSynchronize(d.stream), RADPUL_HIP_MEM_COPY_DEVICE_HOST);
    if (d.list_host.p[0].x != cnt) {  // the same batch, thresholds and spectrum: cannot differ
      log_message(LOG_ERROR, true, "Bounded output re-run emitted %u values, the first run %u.\n", d.list_host.p[0].x,
                  cnt);
      return RADPUL_HIP_CAND_OVERFLOW;
    }
    src = d.list_host.p + 1;
    extra = true;
    d.st.tie_reruns += 1;
    d.st.list_dma_copies += 1;
    d.prev_done = nullptr;
  }
  if (ran_select && d.select_mode && !d.select_forced && o.h_cands_p[0].y <= d.cap / 4) {
    // the thresholds (table floors) rose: the compacting path fits again
    d.select_mode = false;
    d.st.select_exits += 1;
  }
  if (ran_select) d.st.select_batches += 1;
  d.st.candidates += cnt;
  // beyond kcopy entries a DMA copy of the list beats reading it in place
  // (uncached reads over the PCIe BAR) or a second copied prefix
  if (!extra && cnt > (d.fg_out ? d.inplace_max : d.kcopy)) {
    int rc;
    if ((rc = d.list_host.reserve(cnt))) return rc;
    // stream-ordered (a null-stream copy would invalidate another engine's
    // graph capture running in a sibling thread); waits for a batch queued
    // behind this one too, which writes only its own I/O slot
    BRP_HIP_CHECK(memcpy_async(d.list_host.p, o.cands.p + 1, cnt * sizeof(uint2), hipMemcpyDeviceToHost, d.stream),
                  RADPUL_HIP_MEM_COPY_DEVICE_HOST);
    BRP_HIP_CHECK(hipStreamSynchronize(d.stream), RADPUL_HIP_MEM_COPY_DEVICE_HOST);
    src = d.list_host.p;
    d.st.list_dma_copies += 1;
  }
  out.clear();
  out.resize(nb);
  const uint32_t bb = d.bin_bits;
  const uint32_t bin_mask = static_cast<uint32_t>((1ull << bb) - 1u);
  for (uint32_t q = 0; q < cnt; ++q) {
    const uint32_t key = src[q].x;
    const uint32_t k = static_cast<uint32_t>(static_cast<uint64_t>(key) >> (bb + 3)), h = (key >> bb) & 7u;
    if (k >= static_cast<uint32_t>(nb) || h >= static_cast<uint32_t>(kNumHarmonicLevels)) {
      log_message(LOG_ERROR, true,
                  "Candidate %u of %u has key 0x%08x (template %u of %d, level %u; bounded output %d, list %s).\n", q,
                  cnt, key, k, nb, h, ran_select ? 1 : 0, extra ? "copied" : "in place");
      return RADPUL_EVAL;
    }
    float p;
    std::memcpy(&p, &src[q].y, sizeof(float));
    out[k].level[h].push_back(BinPower{key & bin_mask, p});
  }
  for (int k = 0; k < nb; ++k)
    for (int h = 0; h < kNumHarmonicLevels; ++h) {
      std::vector<BinPower>& lv = out[k].level[h];
      std::sort(lv.begin(), lv.end(), [](const BinPower& a, const BinPower& b) { return a.bin < b.bin; });
    }
  return 0;
}

namespace {
// Test hooks check the whole device before they copy: a fault of earlier work
// (any stream) is then reported as such, with the checked build's record of
// the kernel that made it, instead of as a failure of the hook's own copy
// (round 5: an illegal address surfaced at bound_cells' copy).
int device_ok(const char* hook) {
  std::string rep;
  if (hipk::device_check(&rep) == 0) return 0;
  log_message(LOG_ERROR, true, "%s: device fault before this call: %s\n", hook, rep.c_str());
  return RADPUL_HIP_KERNEL_INVOKE;
}
}  // namespace

int HipEngine::power_spectrum(const TemplateInput& t, std::vector<float>& ps_out, uint32_t* n_steps) {
  Impl& d = *impl_;
  if (d.io_busy()) return RADPUL_EMISC;
  BRP_HIP_CHECK(hipSetDevice(d.device), RADPUL_HIP_DEVICE_SET);
  if (int rc = device_ok("power_spectrum")) return rc;
  d.select_io(0);
  const SearchGeometry& g = d.g;
  TemplateDev td{};
  td.p = make_resamp_params(g.nsamples, g.n_unpadded, g.fft_size, g.dt, g.step_inv, t.P, t.tau, t.Psi0);
  td.mu0 = d.mu0s[0];
  td.n_steps = resamp_n_steps(td.p, kSinLut, kCosLut);
  d.h_tmpl.p[0] = td;
  hipStream_t s = d.stream;
  if (!d.fg_in)
    BRP_HIP_CHECK(memcpy_async(d.tmpl.p, d.h_tmpl.p, sizeof(TemplateDev), hipMemcpyHostToDevice, s),
                  RADPUL_HIP_MEM_COPY_HOST_DEVICE);
  std::atomic_thread_fence(std::memory_order_seq_cst);
  if (d.bs) {
    DevBuf<float> full;
    int rc;
    if ((rc = full.alloc(g.fft_size))) return rc;
    BRP_HIP_CHECK(d.bs_template_spectra(1, full.p, nullptr, g.fft_size, g.fft_size), RADPUL_HIP_KERNEL_INVOKE);
    BRP_HIP_CHECK(hipStreamSynchronize(s), RADPUL_HIP_KERNEL_INVOKE);
    if (int rc2 = device_ok("power_spectrum")) return rc2;
    ps_out.resize(g.fft_size);
    BRP_HIP_CHECK(d.copy_out(ps_out.data(), full.p, g.fft_size * sizeof(float)), RADPUL_HIP_MEM_COPY_DEVICE_HOST);
    if (n_steps) *n_steps = d.h_tmpl.p[0].n_steps;
    return 0;
  }
  BRP_HIP_CHECK(d.fft_pass1(1, nullptr), RADPUL_HIP_KERNEL_INVOKE);
  BRP_HIP_CHECK(d.fft_pass2(1), RADPUL_HIP_KERNEL_INVOKE);
  DevBuf<float> full;
  int rc;
  if ((rc = full.alloc(g.fft_size))) return rc;
  BRP_HIP_CHECK(d.fft_pass3(1, full.p, nullptr, g.fft_size, g.fft_size), RADPUL_HIP_KERNEL_INVOKE);
  BRP_HIP_CHECK(hipStreamSynchronize(s), RADPUL_HIP_KERNEL_INVOKE);
  if (int rc2 = device_ok("power_spectrum")) return rc2;
  ps_out.resize(g.fft_size);
  BRP_HIP_CHECK(d.copy_out(ps_out.data(), full.p, g.fft_size * sizeof(float)), RADPUL_HIP_MEM_COPY_DEVICE_HOST);
  if (n_steps) *n_steps = d.h_tmpl.p[0].n_steps;
  return 0;
}

int HipEngine::download_series(std::vector<float>& series) {
  Impl& d = *impl_;
  if (!d.ready || !d.shared_series_valid()) return RADPUL_EMISC;
  BRP_HIP_CHECK(hipSetDevice(d.device), RADPUL_HIP_DEVICE_SET);
  if (int rc = device_ok("download_series")) return rc;
  series.resize(d.g.n_unpadded);
  BRP_HIP_CHECK(d.copy_out(series.data(), d.series_in(), d.g.n_unpadded * sizeof(float)), RADPUL_HIP_MEM_COPY_DEVICE_HOST);
  return 0;
}

int HipEngine::benchmark_stages(const TemplateInput* t, int n, int reps, std::vector<double>& us_per_launch) {
  Impl& d = *impl_;
  if (!d.ready || d.io_busy()) return RADPUL_EMISC;
  d.select_io(0);
  const int nb = std::min(n, d.batch);
  const SearchGeometry& g = d.g;
  // BRP_STAGE_THR_SCALE: scale the chi^2 thresholds (harmonic-sum ablations:
  // a large factor leaves the pruned kernel no exact work)
  const char* ts = std::getenv("BRP_STAGE_THR_SCALE");
  const float thr_scale = ts ? static_cast<float>(std::atof(ts)) : 1.0f;
  for (int k = 0; k < nb; ++k) {
    TemplateDev td{};
    td.p = make_resamp_params(g.nsamples, g.n_unpadded, g.fft_size, g.dt, g.step_inv, t[k].P, t[k].tau, t[k].Psi0);
    td.n_steps = resamp_n_steps(td.p, kSinLut, kCosLut);
    td.mu0 = d.mu0s[0];
    d.h_tmpl.p[k] = td;
    for (int h = 0; h < kNumHarmonicLevels; ++h)
      d.h_thr.p[k * hipk::kHsThrStride + h] = d.g.chi2_thr[h] * thr_scale;
  }
  std::atomic_thread_fence(std::memory_order_seq_cst);
  BRP_HIP_CHECK(d.enqueue(nb), RADPUL_HIP_KERNEL_INVOKE);
  BRP_HIP_CHECK(hipStreamSynchronize(d.stream), RADPUL_HIP_KERNEL_INVOKE);
  us_per_launch.assign(Impl::kNumStages + 1, 0.0);
  for (int st = 0; st <= Impl::kNumStages; ++st) {
    // st == kNumStages: the whole pipeline. Every stage starts from the data of
    // one full run (pass 2 works in place, so repeating it alone drifts the data).
    BRP_HIP_CHECK(d.enqueue(nb), RADPUL_HIP_KERNEL_INVOKE);
    BRP_HIP_CHECK(hipEventRecord(d.ev0, d.stream), RADPUL_HIP_KERNEL_INVOKE);
    for (int r = 0; r < reps; ++r) {
      if (st == Impl::kNumStages) {
        BRP_HIP_CHECK(d.enqueue(nb), RADPUL_HIP_KERNEL_INVOKE);
      } else {
        // the harmonic stage appends to the candidate lists: reset their
        // counters (a 100-byte memset) so every repetition sees the same load
        if (st == Impl::kHarmonic)
          BRP_HIP_CHECK(hipMemsetAsync(d.cands.p, 0, sizeof(uint2), d.stream), RADPUL_HIP_KERNEL_INVOKE);
        BRP_HIP_CHECK(d.enqueue_stage(st, nb), RADPUL_HIP_KERNEL_INVOKE);
      }
    }
    BRP_HIP_CHECK(hipEventRecord(d.ev1, d.stream), RADPUL_HIP_KERNEL_INVOKE);
    trace::range_pop();
    {
      trace::Range wait("brp:batch_wait");
      BRP_HIP_CHECK(hipStreamSynchronize(d.stream), RADPUL_HIP_KERNEL_INVOKE);
    }
    trace::Range decode("brp:batch_decode");
    float ms = 0;
    (void)hipEventElapsedTime(&ms, d.ev0, d.ev1);
    us_per_launch[st] = 1e3 * ms / reps;
  }
  return 0;
}

int HipEngine::bound_cells(int k, std::vector<float>& cells) {
  Impl& d = *impl_;
  if (!d.ready || k < 0 || k >= d.batch || !d.hs_prune || d.hs_cell_shift != 3) return RADPUL_EVAL;
  BRP_HIP_CHECK(hipSetDevice(d.device), RADPUL_HIP_DEVICE_SET);
  if (int rc = device_ok("bound_cells")) return rc;
  cells.resize((d.ps_stride >> 3) + 8);
  BRP_HIP_CHECK(d.copy_out(cells.data(), d.pyr.p + static_cast<size_t>(k) * hipk::hs_pyr_stride(d.ps_stride),
                           cells.size() * sizeof(float)),
                RADPUL_HIP_MEM_COPY_DEVICE_HOST);
  return 0;
}

BackendStats HipEngine::stats() const {
  impl_->settle_whiten(false);
  return impl_->st;
}
int HipEngine::device() const { return impl_->device; }
const FFTPlan3& HipEngine::plan() const { return impl_->plan; }
int HipEngine::batch() const { return impl_->slot_cap(); }

// ------------------------------------------------------------------ Backend
namespace {
class HipBackend final : public Backend {
 public:
  const char* name() const override { return "hip"; }
  int init(int device, int batch) { return eng_.init(device, batch); }
  int setup(const SearchGeometry& g, const SearchOptions& opt, std::vector<float>& series,
            const std::vector<ZapRange>& zaps) override {
    // padding offset mu0 (the padded FFT is corrected to the reference's mean
    // padding by linearity); a whitened series has its DC removed: mu0 = 0, the
    // value the whitening backend itself uses, so all devices compute identical spectra
    double mean = 0.0;
    if (!opt.prewhitened && !opt.white) {  // whitening resets mu0 to 0 (the sum is a 4M-long serial chain)
      for (float v : series) mean += v;
      mean = series.empty() ? 0.0 : mean / series.size();
    }
    if (opt.ps_fp16 && !(opt.white || opt.prewhitened)) {
      log_message(LOG_ERROR, true, "The fp16 power spectrum needs whitening (-W): raw powers overflow fp16.\n");
      return RADPUL_EVAL;
    }
    eng_.set_ps_fp16(opt.ps_fp16);
    int rc = packed_ != nullptr ? eng_.setup_packed(g, *packed_, static_cast<float>(mean))
                                : eng_.setup(g, series, static_cast<float>(mean));
    if (rc == 0 && opt.white) rc = eng_.whiten(opt, zaps, series, 0, !opt.device_series);
    log_message(LOG_DEBUG, true, "HIP device allocations so far: %ld\n", g_device_allocs.load());
    return rc;
  }
  int setup_wu(const SearchGeometry& g, const SearchOptions& opt, WorkUnit& wu,
               const std::vector<ZapRange>& zaps) override {
    // the series stays on the device (or is read back by whiten): upload the payload
    if (!wu.packed.empty() && (opt.white ? opt.device_series : true)) packed_ = &wu;
    const int rc = setup(g, opt, wu.samples, zaps);
    packed_ = nullptr;
    return rc;
  }
  int process(const TemplateInput* t, int n, const float thr[kNumHarmonicLevels],
              std::vector<TemplateCands>& out) override {
    return eng_.process(t, n, thr, out);
  }
  int max_in_flight() const override { return eng_.max_in_flight(); }
  int submit(const TemplateInput* t, int n, const float thr[kNumHarmonicLevels]) override {
    return eng_.submit(t, n, thr, 0);
  }
  int complete(std::vector<TemplateCands>& out) override { return eng_.complete(out); }
  // any HIP backend can take the first
  // backend's whitened series without a host round trip: pipelines on the same
  // device read it in place (adopt_series), other devices get a peer copy over
  // xGMI (setup_peer). BRP_PEER_SERIES=1 forces the copy on one device (tests).
  bool can_setup_from(const Backend& first, const SearchGeometry& g) const override {
    (void)g;
    const auto* src = dynamic_cast<const HipBackend*>(&first);
    return src != nullptr && src != this;
  }
  // -1: not applicable; otherwise the engine's error code (an allocation
  // failure here must still reach the wrapper as a transient resource error)
  int setup_from(const Backend& first, const SearchGeometry& g) override {
    if (!can_setup_from(first, g)) return -1;
    const HipEngine& src = dynamic_cast<const HipBackend&>(first).eng_;
    if (!src.prepared_for(g)) return -1;
    eng_.set_ps_fp16(src.ps_fp16());  // the session's spectrum precision
    const bool force_peer = std::getenv("BRP_PEER_SERIES") != nullptr && std::atoi(std::getenv("BRP_PEER_SERIES")) != 0;
    if (eng_.device() == src.device() && !force_peer) {
      if (!eng_.prepared_for(g)) {  // first pass: allocate (D2D copy)
        const int rc = eng_.setup_peer(src);
        if (rc) return rc;
      }
      return eng_.adopt_series(src);
    }
    return eng_.setup_peer(src);
  }
  int debug_buffers(const TemplateInput& t, std::vector<float>& series, std::vector<float>& ps) override {
    int rc = eng_.download_series(series);
    if (rc == 0) rc = eng_.power_spectrum(t, ps, nullptr);
    return rc;
  }
  int device() const override { return eng_.device(); }
  int warm_up() override { return eng_.warm_up(); }
  int preferred_batch() const override { return eng_.batch(); }
  BackendStats stats() const override { return eng_.stats(); }

 private:
  HipEngine eng_;
  const WorkUnit* packed_ = nullptr;  // setup_wu in progress
};
}  // namespace

std::shared_ptr<void> hip_pin_host(void* p, size_t bytes) {
  if (p == nullptr || bytes == 0 || hipHostRegister(p, bytes, hipHostRegisterDefault) != hipSuccess) {
    (void)hipGetLastError();
    return {};
  }
  return std::shared_ptr<void>(p, [](void* q) { (void)hipHostUnregister(q); });
}

bool hip_backend_supports(const SearchGeometry& g) {
  FFTPlan3 p;
  if (g.nsamples % 2 == 0 && make_fft_plan(g.nsamples / 2, p)) return true;
  return make_bluestein_plan(g.nsamples % 2 ? g.nsamples : g.nsamples / 2, p);  // chirp-z path
}

std::unique_ptr<Backend> make_hip_backend(int device, int batch, int* err) {
  auto b = std::make_unique<HipBackend>();
  int rc = b->init(device, batch);
  if (err) *err = rc;
  if (rc) return nullptr;
  return b;
}

}  // namespace brp
