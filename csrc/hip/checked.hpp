// Checked build (device-side debug mode): `_build.py --checked`
// compiles every source with BRP_CHECKED into the module _brp_checked (and
// bin/einsteinbinary_mi355x_checked). In that build
//   * every kernel launch goes through BRP_LAUNCH: launches are serialised
//     process-wide, each one is followed by a synchronisation of its stream,
//     a look at the runtime's error state, a scan of the guard zones behind
//     every device allocation and a look at the device-side violation record,
//     and a failure is logged with the kernel's name and charged to the call
//     that launched it (launch_status());
//   * global-memory accesses of the kernels go through BRP_LD / BRP_ST /
//     BRP_CHK: the address range must lie inside ONE live device allocation
//     (the registry DevBuf keeps, uploaded to the device before a launch when it
//     changed); a violation is recorded (source line, address, size, block,
//     thread) and the access is skipped, so the checked build never touches
//     memory outside an allocation itself;
//   * each allocation carries a 64 KB guard zone after its end, filled with a
//     pattern: a write past the end at an access that is not instrumented is
//     found by the guard scan after the launch that made it.
// In the product build the macros are the plain accesses and launches
// (identical code). The reference's debugging aids are buffer dumps
// (cuda/app/cuda_utilities.c:283-320) and the !NDEBUG memory tracing of
// demod_binary.c:1126-1176; neither localises a device fault.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <string>

namespace brp {
namespace hipk {

struct ChkRange {
  uint64_t lo, hi;  // [lo, hi): the allocation's requested bytes
  uint64_t gend;    // end of its guard zone
};
constexpr int kChkMaxRanges = 1024;
constexpr uint32_t kChkGuardBytes = 64u * 1024u;
constexpr uint32_t kChkGuardWord = 0xA5A5A5A5u;

// test-only injected out-of-bounds accesses (BRP_CHECKED_INJECT=<name>): the
// instrumented kernel forms an index just past its buffer, the check records
// it and skips the access
enum ChkInject : uint32_t {
  kInjNone = 0,
  kInjHsCells = 1,    // hs_cells_kernel: one cell store past the cell buffer
  kInjPass1 = 2,      // pass-1 gather: one series read past the series
  kInjPass3 = 3,      // pass 3: one spectrum store past the spectrum
  kInjHsPruned = 4,   // hs_pruned_kernel: one bound-cell read past the cells
};

// device-resident state of the checked build (one per process)
struct ChkDev {
  uint32_t n_ranges;
  uint32_t inject;
  uint32_t fault;     // 0: clean; first violation's record below
  uint32_t line;      // source line of the access (0: guard zone)
  uint64_t addr;
  uint32_t bytes;
  uint32_t is_store;
  uint32_t block_x, block_y, thread;
  uint32_t pad;
  ChkRange r[kChkMaxRanges];  // sorted by lo, non-overlapping
};

// ---- host side (csrc/engine/checked.cpp; no-ops in the product build)
bool checked_build();
void chk_register(const void* p, size_t bytes, size_t alloc_bytes);
void chk_unregister(const void* p);
// extra bytes an allocation of `bytes` gets (its guard zone; 0 in the product build)
size_t chk_guard_bytes();
// the guard zone of a fresh allocation (pattern fill)
hipError_t chk_fill_guard(void* p, size_t bytes);
void chk_before_launch(hipStream_t s);
void chk_after_launch(const char* kernel, hipStream_t s);
// launch status of the launcher that just ran: the runtime's error, or the
// checked build's violation report of this thread's last launches
hipError_t chk_take_error();
// device-wide check: hipDeviceSynchronize + hipGetLastError (+ guard scan and
// the pending violation record in the checked build). 0 and an empty report
// when clean.
int device_check(std::string* report);
// the host side of an engine copy is pinned (or host-visible device) memory,
// never pageable memory the runtime would pin in place per copy (checked
// build: a report otherwise; round-5 fault, profiles/fault_r6.txt)
void chk_host_copy(const void* host, size_t bytes);
// per-translation-unit device pointer binding (checked build)
using ChkBinder = hipError_t (*)(ChkDev*);
int chk_register_binder(ChkBinder b);
// guard scan kernel (checked.hip)
hipError_t launch_guard_scan(ChkDev* dev, uint32_t n_ranges, hipStream_t s);

#ifdef BRP_CHECKED
#define BRP_LAUNCH(K, G, B, SH, S, ...)                 \
  do {                                                  \
    ::brp::hipk::chk_before_launch(S);                  \
    hipLaunchKernelGGL(K, G, B, SH, S, __VA_ARGS__);    \
    ::brp::hipk::chk_after_launch(#K, S);               \
  } while (0)
#else
#define BRP_LAUNCH(K, G, B, SH, S, ...) hipLaunchKernelGGL(K, G, B, SH, S, __VA_ARGS__)
#endif

inline hipError_t launch_status() {
#ifdef BRP_CHECKED
  const hipError_t e = hipGetLastError();
  const hipError_t c = chk_take_error();
  return e != hipSuccess ? e : c;
#else
  return hipGetLastError();
#endif
}

#if defined(__HIP__) && defined(BRP_CHECKED)
namespace {
// this translation unit's view of the process's ChkDev (set by the binder)
__device__ ChkDev* g_chk_dev = nullptr;
hipError_t chk_bind_this_tu(ChkDev* p) { return hipMemcpyToSymbol(HIP_SYMBOL(g_chk_dev), &p, sizeof(p)); }
[[maybe_unused]] const int g_chk_tu_registered = chk_register_binder(&chk_bind_this_tu);

// inlined, as chk_addr: an out-of-line call in divergent code before a
// wave-aggregated emit (ballot, leader atomic, broadcast) left holes in the
// candidate list of the select path (round 6, the first checked build)
__device__ __forceinline__ void chk_record(ChkDev* c, uint64_t a, uint32_t bytes, uint32_t line, bool st) {
  if (atomicCAS(&c->fault, 0u, 1u) != 0u) return;
  c->line = line;
  c->addr = a;
  c->bytes = bytes;
  c->is_store = st ? 1u : 0u;
  c->block_x = blockIdx.x;
  c->block_y = blockIdx.y;
  c->thread = threadIdx.x;
  __threadfence_system();
}

// [p, p + bytes) inside one live allocation (binary search of the sorted ranges)
__device__ __forceinline__ bool chk_addr(const void* p, uint32_t bytes, uint32_t line, bool st) {
  ChkDev* c = g_chk_dev;
  if (c == nullptr) return true;
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  int lo = 0, hi = static_cast<int>(c->n_ranges) - 1, hit = -1;
  while (lo <= hi) {
    const int mid = (lo + hi) >> 1;
    if (c->r[mid].lo <= a) {
      hit = mid;
      lo = mid + 1;
    } else {
      hi = mid - 1;
    }
  }
  if (hit >= 0 && a + bytes <= c->r[hit].hi) return true;
  chk_record(c, a, bytes, line, st);
  return false;
}

__device__ __forceinline__ bool chk_injected(uint32_t site) {
  const ChkDev* c = g_chk_dev;
  return c != nullptr && c->inject == site && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0;
}
}  // namespace

template <typename T>
__device__ __forceinline__ T chk_ld(const T* p, uint32_t line) {
  return chk_addr(p, sizeof(T), line, false) ? *p : T{};
}
template <typename T, typename V>
__device__ __forceinline__ void chk_st(T* p, const V& v, uint32_t line) {
  if (chk_addr(p, sizeof(T), line, true)) *p = v;
}
// load / store / range check of an instrumented global access
#define BRP_LD(p) (::brp::hipk::chk_ld((p), __LINE__))
#define BRP_ST(p, v) (::brp::hipk::chk_st((p), (v), __LINE__))
#define BRP_CHK(p, bytes) (::brp::hipk::chk_addr((p), (bytes), __LINE__, false))
// `bad` instead of `idx` for the one thread the test-only injection of `site`
// picks (an index just past the buffer's end: inside its guard zone, never in
// another allocation)
#define BRP_INJECT_AT(idx, bad, site) (::brp::hipk::chk_injected(site) ? (bad) : (idx))
#else
#define BRP_LD(p) (*(p))
#define BRP_ST(p, v) (*(p) = (v))
#define BRP_CHK(p, bytes) true
#define BRP_INJECT_AT(idx, bad, site) (idx)
#endif

}  // namespace hipk
}  // namespace brp
