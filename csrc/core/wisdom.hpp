// Plan wisdom: measured launch settings per (GPU architecture, FFT size), the
// counterpart of the reference's FFTW wisdom (demod_binary_fft_fftw.c:65-69,
// debian/extra/create_wisdomf_eah_brp.sh). tools/tune_plan.py measures the
// candidates on the target GPU and writes data/wisdom/mi355x.json; the HIP
// engine applies the entry of its (arch, M) at setup; BRP_PERSIST overrides it.
//
// Format (JSON): {"entries": [{"arch": "gfx950", "M": 6291456,
//                  "persist_per_cu": 4, "batch": 1, "pipelines": 3, ...}, ...]}
#pragma once

#include <cstdint>
#include <string>

namespace brp {

struct PlanWisdom {
  bool found = false;
  int persist_per_cu = -1;  // pass-2 persistent workgroups per CU
  int batch = -1;           // templates per device batch
  int pipelines = -1;       // pipelines per GPU
};

// $BRP_WISDOM, else data/wisdom/mi355x.json beside the directory holding the
// binary that contains this code (bin/ or the Python package directory).
std::string wisdom_path();

// Entry for (arch, M) in the file at `path`; found == false if the file or the
// entry is missing or malformed. `arch` is compared up to the first ':'
// (gcnArchName "gfx950:sramecc+:xnack-" matches "gfx950").
PlanWisdom load_wisdom(const std::string& path, const std::string& arch, uint32_t M);

}  // namespace brp
