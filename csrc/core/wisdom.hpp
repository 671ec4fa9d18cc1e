// Plan wisdom: measured launch settings per (GPU architecture, FFT size), the
// counterpart of the reference's FFTW wisdom (demod_binary_fft_fftw.c:65-69,
// debian/extra/create_wisdomf_eah_brp.sh). tools/tune_plan.py measures the
// candidates on the target GPU and writes data/wisdom/mi355x.json; the HIP
// engine applies the entry of its (arch, M) at setup. Environment variables
// (BRP_PERSIST, BRP_FFT2, BRP_HS_STAGE, BRP_HS_TILE) override it.
//
// Format (JSON): {"entries": [{"arch": "gfx950", "M": 6291456,
//                  "persist_per_cu": 4, "fft_passes": 3, "hs_stage": 0, "hs_tile": 1008,
//                  "batch": 1, "pipelines": 3, ...}, ...]}
#pragma once

#include <cstdint>
#include <string>

namespace brp {

struct PlanWisdom {
  bool found = false;
  int persist_per_cu = -1;  // pass-2 persistent workgroups per CU
  int fft_passes = -1;      // 3 or 2 (two-pass template FFT)
  int hs_stage = -1;        // harmonics staged in LDS by the harmonic sum
  int hs_tile = -1;         // harmonic-sum bins per workgroup
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
