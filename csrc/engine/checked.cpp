// Host side of the checked build (csrc/hip/checked.hpp): the registry of live
// device allocations, its device copy, serialised and verified launches, and
// device_check(). In the product build only device_check() does work
// (hipDeviceSynchronize + hipGetLastError) and the rest are no-ops.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../core/log.hpp"
#include "../hip/checked.hpp"

namespace brp {
namespace hipk {

namespace {
std::vector<ChkBinder>& binders() {
  static std::vector<ChkBinder> b;
  return b;
}
}  // namespace

int chk_register_binder(ChkBinder b) {
  binders().push_back(b);
  return static_cast<int>(binders().size());
}

#ifdef BRP_CHECKED

namespace {

struct Registry {
  std::mutex mu;                                         // ranges, version, report
  std::map<uint64_t, std::pair<uint64_t, uint64_t>> ranges;  // lo -> (hi, guard end)
  uint64_t version = 1, uploaded = 0;
  uint32_t n_uploaded = 0;                               // ranges in the device copy
  ChkDev* dev = nullptr;                                 // device copy (hipMalloc)
  bool bound = false;
  uint32_t inject = kInjNone;
  std::recursive_mutex launch_mu;                        // serialised launches
  std::string report;                                    // first unreported violation
  std::atomic<int> pending{0};
};

Registry& reg() {
  static Registry* r = new Registry;  // never destroyed: allocations may outlive static teardown
  return *r;
}

thread_local hipError_t t_launch_error = hipSuccess;

uint32_t inject_from_env() {
  const char* e = std::getenv("BRP_CHECKED_INJECT");
  if (e == nullptr) return kInjNone;
  const std::string s = e;
  if (s == "hs_cells") return kInjHsCells;
  if (s == "pass1") return kInjPass1;
  if (s == "pass3") return kInjPass3;
  if (s == "hs_pruned") return kInjHsPruned;
  return kInjNone;
}

// device state allocated and bound to every translation unit (once)
hipError_t ensure_bound(Registry& r) {
  if (r.bound) return hipSuccess;
  hipError_t e = hipMalloc(reinterpret_cast<void**>(&r.dev), sizeof(ChkDev));
  if (e != hipSuccess) return e;
  if ((e = hipMemset(r.dev, 0, sizeof(ChkDev))) != hipSuccess) return e;
  r.inject = inject_from_env();
  if ((e = hipMemcpy(&r.dev->inject, &r.inject, sizeof(uint32_t), hipMemcpyHostToDevice)) != hipSuccess) return e;
  for (ChkBinder b : binders())
    if ((e = b(r.dev)) != hipSuccess) return e;
  r.bound = true;
  if (r.inject != kInjNone)
    log_message(LOG_WARN, true, "checked build: injected out-of-bounds access %u (BRP_CHECKED_INJECT)\n", r.inject);
  return hipSuccess;
}

// the registry's ranges into the device copy (caller holds launch_mu; the
// device is idle: every launch before this one was synchronised)
hipError_t upload(Registry& r) {
  std::vector<ChkRange> v;
  uint64_t ver;
  {
    std::lock_guard<std::mutex> lk(r.mu);
    ver = r.version;
    if (ver == r.uploaded) return hipSuccess;
    for (const auto& kv : r.ranges) {
      if (v.size() == static_cast<size_t>(kChkMaxRanges)) break;
      v.push_back(ChkRange{kv.first, kv.second.first, kv.second.second});
    }
    if (r.ranges.size() > static_cast<size_t>(kChkMaxRanges))
      log_message(LOG_WARN, true, "checked build: %zu live allocations, only %d checked\n", r.ranges.size(),
                  kChkMaxRanges);
  }
  const uint32_t n = static_cast<uint32_t>(v.size());
  hipError_t e = hipDeviceSynchronize();
  if (e == hipSuccess && n) e = hipMemcpy(r.dev->r, v.data(), n * sizeof(ChkRange), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(&r.dev->n_ranges, &n, sizeof(n), hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    std::lock_guard<std::mutex> lk(r.mu);
    r.uploaded = ver;
    r.n_uploaded = n;
  }
  return e;
}

// the device's violation record (and the guard scan) after synchronised work;
// returns a report, empty when clean, and clears the record
std::string collect(Registry& r, hipStream_t s, const char* kernel) {
  if (!r.bound) return {};
  // the device copy of the ranges first: allocations freed since the last
  // launch (a hook's scratch buffer) must not be scanned
  hipError_t e = upload(r);
  if (e == hipSuccess) e = launch_guard_scan(r.dev, r.n_uploaded, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    char buf[256];
    std::snprintf(buf, sizeof(buf), "checked: guard scan after %s failed: %s", kernel, hipGetErrorName(e));
    return buf;
  }
  ChkDev head;
  e = hipMemcpy(&head, r.dev, offsetof(ChkDev, r), hipMemcpyDeviceToHost);
  if (e != hipSuccess || head.fault == 0) return {};
  // which allocation the address is nearest to (below it)
  uint64_t lo = 0, hi = 0;
  {
    std::lock_guard<std::mutex> lk(r.mu);
    auto it = r.ranges.upper_bound(head.addr);
    if (it != r.ranges.begin()) {
      --it;
      lo = it->first;
      hi = it->second.first;
    }
  }
  char buf[512];
  if (head.line == 0) {
    std::snprintf(buf, sizeof(buf),
                  "checked: kernel %s wrote past an allocation: guard word at 0x%" PRIx64
                  " (allocation [0x%" PRIx64 ", 0x%" PRIx64 "), %" PRIu64 " bytes past its end)",
                  kernel, head.addr, lo, hi, head.addr - hi);
  } else {
    std::snprintf(buf, sizeof(buf),
                  "checked: kernel %s: out-of-bounds %s of %u bytes at 0x%" PRIx64
                  " (source line %u, block (%u, %u), thread %u; nearest allocation below: [0x%" PRIx64 ", 0x%" PRIx64
                  ")%s)",
                  kernel, head.is_store ? "store" : "load", head.bytes, head.addr, head.line, head.block_x,
                  head.block_y, head.thread, lo, hi, (lo && head.addr >= hi) ? ", past its end" : "");
  }
  const uint32_t zero = 0;
  (void)hipMemcpy(&r.dev->fault, &zero, sizeof(zero), hipMemcpyHostToDevice);
  // a guard word that was hit stays reported until the allocation is freed:
  // refill it
  if (head.line == 0 && hi) {
    std::lock_guard<std::mutex> lk(r.mu);
    auto it = r.ranges.find(lo);
    if (it != r.ranges.end())
      (void)hipMemset(reinterpret_cast<void*>(hi), 0xA5, static_cast<size_t>(it->second.second - hi));
  }
  return buf;
}

void set_report(Registry& r, const std::string& s) {
  log_message(LOG_ERROR, true, "%s\n", s.c_str());
  std::lock_guard<std::mutex> lk(r.mu);
  if (r.report.empty()) r.report = s;
  r.pending.store(1);
}

}  // namespace

bool checked_build() { return true; }

size_t chk_guard_bytes() { return kChkGuardBytes; }

hipError_t chk_fill_guard(void* p, size_t bytes) {
  return hipMemset(static_cast<char*>(p) + bytes, 0xA5, kChkGuardBytes);
}

void chk_register(const void* p, size_t bytes, size_t alloc_bytes) {
  Registry& r = reg();
  std::lock_guard<std::mutex> lk(r.mu);
  const uint64_t lo = reinterpret_cast<uint64_t>(p);
  r.ranges[lo] = {lo + bytes, lo + alloc_bytes};
  ++r.version;
}

void chk_unregister(const void* p) {
  Registry& r = reg();
  // not while a launch or guard scan of this process may read the range
  std::lock_guard<std::recursive_mutex> lk0(r.launch_mu);
  std::lock_guard<std::mutex> lk(r.mu);
  r.ranges.erase(reinterpret_cast<uint64_t>(p));
  ++r.version;
}

void chk_before_launch(hipStream_t s) {
  Registry& r = reg();
  r.launch_mu.lock();  // released by chk_after_launch (BRP_LAUNCH pairs them)
  // a launch being captured into a graph runs later: no device-wide work now
  // (a synchronisation would invalidate the capture)
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) return;
  hipError_t e = ensure_bound(r);
  if (e == hipSuccess) e = upload(r);
  if (e != hipSuccess) {
    set_report(r, std::string("checked: registry upload failed: ") + hipGetErrorName(e));
    t_launch_error = e;
  }
}

void chk_after_launch(const char* kernel, hipStream_t s) {
  Registry& r = reg();
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) {
    r.launch_mu.unlock();  // captured: checked when the graph runs (graphs are off by default)
    return;
  }
  const hipError_t le = hipPeekAtLastError();
  hipError_t e = hipStreamSynchronize(s);
  std::string rep;
  if (le != hipSuccess || e != hipSuccess) {
    char buf[256];
    std::snprintf(buf, sizeof(buf), "checked: kernel %s: %s", kernel,
                  hipGetErrorName(le != hipSuccess ? le : e));
    rep = buf;
  } else {
    rep = collect(r, s, kernel);
  }
  if (!rep.empty()) {
    set_report(r, rep);
    if (t_launch_error == hipSuccess) t_launch_error = le != hipSuccess ? le : (e != hipSuccess ? e : hipErrorLaunchFailure);
  }
  r.launch_mu.unlock();
}

void chk_host_copy(const void* host, size_t bytes) {
  hipPointerAttribute_t at{};
  const hipError_t e = hipPointerGetAttributes(&at, host);
  if (e != hipSuccess) (void)hipGetLastError();
  const bool ok = e == hipSuccess && (at.type == hipMemoryTypeHost || at.type == hipMemoryTypeDevice ||
                                      at.type == hipMemoryTypeManaged);
  if (ok) return;
  char buf[256];
  std::snprintf(buf, sizeof(buf), "checked: a host copy of %zu bytes uses pageable memory at %p", bytes, host);
  set_report(reg(), buf);
}

hipError_t chk_take_error() {
  const hipError_t e = t_launch_error;
  t_launch_error = hipSuccess;
  return e;
}

int device_check(std::string* report) {
  Registry& r = reg();
  std::lock_guard<std::recursive_mutex> lk(r.launch_mu);
  std::string rep;
  hipError_t e = hipDeviceSynchronize();
  const hipError_t le = hipGetLastError();
  if (e != hipSuccess || le != hipSuccess) {
    rep = std::string("device check: ") + hipGetErrorName(e != hipSuccess ? e : le);
  } else if (r.bound) {
    rep = collect(r, nullptr, "(device check)");
  }
  {
    std::lock_guard<std::mutex> lk2(r.mu);
    if (!r.report.empty()) {
      rep = r.report + (rep.empty() ? "" : "; then " + rep);
      r.report.clear();
    }
    r.pending.store(0);
  }
  if (report) *report = rep;
  return rep.empty() ? 0 : 1;
}

#else  // product build

bool checked_build() { return false; }
size_t chk_guard_bytes() { return 0; }
hipError_t chk_fill_guard(void*, size_t) { return hipSuccess; }
void chk_register(const void*, size_t, size_t) {}
void chk_unregister(const void*) {}
void chk_before_launch(hipStream_t) {}
void chk_after_launch(const char*, hipStream_t) {}
hipError_t chk_take_error() { return hipSuccess; }
void chk_host_copy(const void*, size_t) {}

int device_check(std::string* report) {
  const hipError_t e = hipDeviceSynchronize();
  const hipError_t le = hipGetLastError();
  std::string rep;
  if (e != hipSuccess || le != hipSuccess) rep = std::string("device check: ") + hipGetErrorName(e != hipSuccess ? e : le);
  if (report) *report = rep;
  return rep.empty() ? 0 : 1;
}

#endif

}  // namespace hipk
}  // namespace brp
