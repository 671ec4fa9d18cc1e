#include "trace.hpp"

#include <dlfcn.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>

#include "log.hpp"

namespace brp {
namespace trace {
namespace {

struct Roctx {
  int (*push)(const char*) = nullptr;
  int (*pop)() = nullptr;
  void (*mark)(const char*) = nullptr;
  bool on = false;
};

const Roctx& roctx() {
  static Roctx r;
  static std::once_flag once;
  std::call_once(once, [] {
    const char* env = std::getenv("BRP_ROCTX");
    if (!env || !*env || std::strcmp(env, "0") == 0) return;
    const char* libs[] = {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4",
                          "libroctx64.so"};
    void* h = nullptr;
    for (const char* l : libs)
      if ((h = dlopen(l, RTLD_NOW | RTLD_GLOBAL))) break;
    if (!h) {
      log_message(LOG_WARN, true, "BRP_ROCTX set but no roctx library could be loaded: %s\n", dlerror());
      return;
    }
    r.push = reinterpret_cast<int (*)(const char*)>(dlsym(h, "roctxRangePushA"));
    r.pop = reinterpret_cast<int (*)()>(dlsym(h, "roctxRangePop"));
    r.mark = reinterpret_cast<void (*)(const char*)>(dlsym(h, "roctxMarkA"));
    r.on = r.push && r.pop;
    if (r.on) log_message(LOG_DEBUG, true, "roctx ranges enabled.\n");
  });
  return r;
}

}  // namespace

bool enabled() { return roctx().on; }

void range_push(const char* name) {
  const Roctx& r = roctx();
  if (r.on) r.push(name);
}

void range_pop() {
  const Roctx& r = roctx();
  if (r.on) r.pop();
}

void mark(const char* name) {
  const Roctx& r = roctx();
  if (r.on && r.mark) r.mark(name);
}

namespace {
const auto g_t0 = std::chrono::steady_clock::now();  // static init: ~process start
}  // namespace

void phase(const char* name) {
  static const bool on = [] {
    const char* e = std::getenv("BRP_PHASES");
    return e && *e && std::strcmp(e, "0") != 0;
  }();
  mark(name);
  if (!on) return;
  static std::mutex mu;
  static double prev = 0.0;
  std::lock_guard<std::mutex> lk(mu);
  const double t = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - g_t0).count();
  // wall-clock stamp too, so a caller timing the whole process can split off
  // what lies before static initialisation and after the last phase (exit)
  const double epoch_ms =
      std::chrono::duration<double, std::milli>(std::chrono::system_clock::now().time_since_epoch()).count();
  std::fprintf(stderr, "[phase] %-28s t=%8.1f ms  +%7.1f ms  epoch_ms=%.3f\n", name, t, t - prev, epoch_ms);
  prev = t;
}

}  // namespace trace
}  // namespace brp
