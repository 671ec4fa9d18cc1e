// Low-level MI355X engine (used by the HIP backend, the Python bindings and tests).
#pragma once

#include <hip/hip_runtime.h>

#include <vector>

#include "../hip/fft_plan.hpp"
#include "backend.hpp"

namespace brp {

class HipEngine {
 public:
  HipEngine();
  ~HipEngine();
  HipEngine(const HipEngine&) = delete;
  HipEngine& operator=(const HipEngine&) = delete;

  int init(int device, int batch);
  // allocate per-WU buffers, upload the series; mu0 = reference level
  // subtracted before the FFT (keeps the padding correction well conditioned)
  int setup(const SearchGeometry& g, const std::vector<float>& series, float mu0);
  // the same from the WU's stored payload (WorkUnit::packed): n/2 bytes cross
  // PCIe instead of 4n and the device unpacks them (bit-identical floats)
  int setup_packed(const SearchGeometry& g, const WorkUnit& wu, float mu0);
  int upload_series(const std::vector<float>& series, float mu0);
  // Re-setup for the next pass over the same geometry from `src`'s (whitened)
  // series: `src` and this engine share a device, have the same number of WU
  // slots, and this engine was set up before. The pipeline reads `src`'s series in place (one copy in the
  // Infinity Cache for all pipelines; `src` must outlive the search pass), or
  // copies it device to device with BRP_SHARE_SERIES=0. setup(), load_slot()
  // and whiten() return to the engine's own buffer. RADPUL_EVAL when not applicable.
  int adopt_series(const HipEngine& src);
  // Set up from `src`'s prepared (whitened) series, device to device: a
  // hipMemcpyPeer over xGMI when `src` is on another device, a D2D copy on the
  // same one. Allocates like setup() on first use. No host round trip.
  int setup_peer(const HipEngine& src);
  // Multi-WU batching: the series buffer holds `k` work units of the same
  // shape (set before setup(); setup() fills slot 0, load_slot() the others).
  // Templates pick their slot with TemplateInput::wu.
  int set_slots(uint32_t k);
  // config 5: store the power spectrum as fp16 (halves the pass-3 write and the
  // harmonic-sum reads; the sums stay fp32 in the reference order)
  void set_ps_fp16(bool on);
  bool ps_fp16() const;
  uint32_t slots() const;
  int load_slot(uint32_t k, const std::vector<float>& series, float mu0);
  // whitening + zapping of one slot on the device; `series` (that slot's raw
  // data) receives the whitened data
  int whiten(const SearchOptions& opt, const std::vector<ZapRange>& zaps, std::vector<float>& series,
             uint32_t slot = 0, bool copy_back = true);
  // set up (buffers, plan, graphs) for this geometry with one WU slot
  bool prepared_for(const SearchGeometry& g) const;
  // set up for this geometry with any number of slots (multi-WU batching)
  bool ready_for(const SearchGeometry& g) const;
  int process(const TemplateInput* t, int n, const float thr[kNumHarmonicLevels], std::vector<TemplateCands>& out);
  // per-template thresholds thr[i * thr_stride + h] (thr_stride 0: shared)
  int process(const TemplateInput* t, int n, const float* thr, int thr_stride, std::vector<TemplateCands>& out);
  // Pipelined form of process(): submit() launches one batch (n <= batch())
  // and returns at once; complete() waits for the oldest submitted batch and
  // decodes its candidates. Up to max_in_flight() batches may be submitted
  // before the first complete(); process() and the test hooks need none
  // outstanding.
  int submit(const TemplateInput* t, int n, const float* thr, int thr_stride);
  int complete(std::vector<TemplateCands>& out);
  int max_in_flight() const;
  // test hooks
  int power_spectrum(const TemplateInput& t, std::vector<float>& ps, uint32_t* n_steps);
  // the (whitened) series of slot 0 as the templates read it
  int download_series(std::vector<float>& series);
  // the pruned harmonic sum's 8-bin bound cells of template k of the last
  // batch ((ps_stride >> 3) + 8 entries)
  int bound_cells(int k, std::vector<float>& cells);
  // the first work's one-time costs ahead of it (code objects, copy kernels, stage)
  int warm_up();
  // time each pipeline stage (prologue, pass1, pass2, pass3, harmonic, epilogue,
  // whole batch) over `reps` back-to-back launches on one batch; microseconds
  int benchmark_stages(const TemplateInput* t, int n, int reps, std::vector<double>& us_per_launch);

  BackendStats stats() const;
  int device() const;
  int batch() const;
  const FFTPlan3& plan() const;

 private:
  int setup_impl(const SearchGeometry& g, const float* host_series, const float* dev_series, int src_device,
                 float mu0, const WorkUnit* packed = nullptr);
  int upload_series0(const float* host, const float* dev_src, int src_device, const WorkUnit* packed = nullptr);
  struct Impl;
  Impl* impl_;
};

}  // namespace brp
