// Guard-zone scan of the checked build (checked.hpp): after every launch, one
// workgroup per registered allocation reads the 64 KB behind its requested
// bytes and records the first word that lost the fill pattern. Empty in the
// product build.
#include "checked.hpp"

namespace brp {
namespace hipk {

#ifdef BRP_CHECKED
namespace {

__global__ void __launch_bounds__(256) guard_scan_kernel(ChkDev* c) {
  const ChkRange rg = c->r[blockIdx.x];
  const uint64_t g0 = (rg.hi + 3) & ~3ull;  // first whole guard word
  const uint64_t n = (rg.gend - g0) / 4;
  const uint32_t* w = reinterpret_cast<const uint32_t*>(g0);
  for (uint64_t i = threadIdx.x; i < n; i += 256) {
    if (w[i] != kChkGuardWord && atomicCAS(&c->fault, 0u, 1u) == 0u) {
      c->line = 0;
      c->addr = g0 + 4 * i;
      c->bytes = 4;
      c->is_store = 1;
      c->block_x = blockIdx.x;
      c->block_y = 0;
      c->thread = threadIdx.x;
      __threadfence_system();
    }
  }
}

}  // namespace

hipError_t launch_guard_scan(ChkDev* dev, uint32_t n_ranges, hipStream_t s) {
  if (n_ranges == 0) return hipSuccess;
  hipLaunchKernelGGL(guard_scan_kernel, dim3(n_ranges), dim3(256), 0, s, dev);
  return hipGetLastError();
}
#else
hipError_t launch_guard_scan(ChkDev*, uint32_t, hipStream_t) { return hipSuccess; }
#endif

}  // namespace hipk
}  // namespace brp
