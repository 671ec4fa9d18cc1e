// Search geometry (derived bin ranges / thresholds) and the candidate table.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "formats.hpp"

namespace brp {

// User variables of the search (reference User_Variables, demod_binary.c:89-104)
// with the reference defaults (:203-215).
struct SearchOptions {
  float f0 = 250.0f;        // -f  max fundamental frequency [Hz]
  float padding = 1.0f;     // -P  frequency over-resolution factor
  float fA = 0.04f;         // -A  overall false-alarm probability
  uint32_t window = 1000;   // -B  running-median window [bins]
  bool white = false;       // -W  whitening + RFI zapping
  bool debug = false;       // -z
  int device = -1;          // -D  GPU ordinal (auto if < 0)
  std::string inputfile, outputfile, templatebank, checkpointfile, zaplistfile;
  // MI355X extensions (not part of the BOINC command line)
  int batch = 0;            // templates per device batch (0 = auto)
  bool use_cpu = false;     // CPU golden backend instead of HIP
  bool prewhitened = false; // series already whitened by another backend (DC removed)
  bool ps_fp16 = false;     // store the power spectrum as fp16 (config 5; needs -W)
  bool device_series = false;  // the whitened series is only needed on the device (no copy back)
  std::string dump_dir;     // with -z: text dumps of intermediate buffers (reference dumpFloatBufferToTextFile)
};

// Everything derived from the WU header + options (demod_binary.c:778-782,
// 1086-1106, 1157-1165, hs_cpu.c:36).
struct SearchGeometry {
  uint32_t n_unpadded = 0;          // samples in the WU
  uint32_t nsamples = 0;            // padded FFT length N
  uint32_t fft_size = 0;            // N/2 + 1 (round-half-up)
  uint32_t window_2 = 0;            // half running-median window
  uint32_t fundamental_idx_hi = 0;  // first bin beyond the searched fundamentals
  uint32_t harmonic_idx_hi = 0;     // first bin beyond the searched 16th harmonics
  uint32_t nr_pages = 0;            // dirty-page count (statistics)
  float t_obs = 0;                  // padded observation time [s] (float, as used for bins)
  double t_obs_d = 0;               // same in double (output frequencies, zapping)
  float dt = 0;                     // sample time [s]
  float step_inv = 0;               // 1/dt
  float prob = 0;                   // single-bin false-alarm probability
  float chi2_thr[kNumHarmonicLevels] = {0};  // 0.5*Qinv(prob, 2*2^h)
};

int derive_geometry(const DDHeader& h, const SearchOptions& opt, SearchGeometry& g);

// One device-reported candidate bin (above the device threshold) of one level.
struct BinPower {
  uint32_t bin;
  float power;
};

// The 5 x 100 candidate table with the reference's sequential insertion
// semantics (demod_binary.c:1310-1397): keep per level the 100 best distinct
// f0 bins by power, each tagged with the first template reaching that power.
class CandidateTable {
 public:
  CandidateTable() { reset(); }
  void reset();
  CPCand* data() { return c_; }
  const CPCand* data() const { return c_; }
  // Smallest power kept on level h (100th entry; 0 for an empty slot).
  double floor_power(int h) const { return c_[h * kCandPerLevel + kCandPerLevel - 1].power; }
  // thrA[h] = fmaxf(100th power, chi2 threshold) (demod_binary.c:1268-1282)
  void thresholds(const float chi2_thr[kNumHarmonicLevels], float thr[kNumHarmonicLevels]) const;
  // Offer the above-threshold bins of ONE template on level h, in ascending
  // bin order. `thr` is thrA[h] computed at the start of this template.
  // Returns the number of table updates.
  int apply_level(int h, const BinPower* bins, size_t n, float thr, float P, float tau, float Psi0);
  // Associative merge used for sharded/batched runs:
  // top-100 distinct bins by power, ties broken by table order.
  void merge(const CandidateTable& other);

 private:
  void insert_sorted(int h, int store_idx, uint32_t f0, float power, float P, float tau, float Psi0);
  CPCand c_[kCandTotal];
};

}  // namespace brp
