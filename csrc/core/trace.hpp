// roctx ranges for rocprofv3 --marker-trace. The reference
// traces by logging launch geometry (cuda/app/demod_binary_cuda.cu:435) and
// device memory after each setup phase (demod_binary.c:1126-1147); here host
// phases (setup / batch launch / wait / decode / checkpoint / output) become
// named ranges on the profiler timeline next to the kernels.
//
// Off unless BRP_ROCTX=1; the roctx library is dlopen()ed then, so the
// framework has no link-time dependency on the profiler SDK.
#pragma once

namespace brp {
namespace trace {

bool enabled();
void range_push(const char* name);
void range_pop();
void mark(const char* name);
// Process phase timeline (BRP_PHASES=1): "name" at milliseconds since process
// start, and since the previous phase, to stderr; also a roctx mark.
void phase(const char* name);

struct Range {
  explicit Range(const char* name) : on_(enabled()) {
    if (on_) range_push(name);
  }
  ~Range() {
    if (on_) range_pop();
  }
  Range(const Range&) = delete;
  Range& operator=(const Range&) = delete;

 private:
  bool on_;
};

}  // namespace trace
}  // namespace brp
