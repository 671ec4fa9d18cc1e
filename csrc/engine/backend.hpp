// Compute-backend interface of the search driver (the reference selects its
// backend at link time: set_up_/run_/tear_down_{resampling,fft,harmonic_summing},
// demod_binary.c:64-81). Here a backend owns the whole per-WU device state and
// processes *batches* of templates, returning the above-threshold bins of every
// template; the driver applies them to the candidate table in template order.
#pragma once

#include <deque>
#include <memory>
#include <string>
#include <vector>

#include "../core/io.hpp"
#include "../core/search_core.hpp"

namespace brp {

struct TemplateInput {
  float P, tau, Psi0;
  uint32_t wu = 0;  // work-unit slot (multi-WU batching)
};

struct TemplateCands {
  std::vector<BinPower> level[kNumHarmonicLevels];  // ascending bins
};

struct BackendStats {
  // Sum over batches of the time from the previous completion on the same
  // stream to this batch's completion event, counted only while batches are
  // queued back to back (an idle stream restarts the chain): the busy span of
  // the stream, not kernel time (rocprofv3 kernel traces give that).
  double busy_span_ms = 0;
  double whiten_ms = 0;      // device time of the whitening step
  uint64_t templates = 0;
  uint64_t batches = 0;
  uint64_t overflow_reruns = 0;   // batches re-run with the bounded output after a list overflow
  uint64_t tie_reruns = 0;        // batches whose bounded output overflowed too (ties at a 100th place): re-run into a list sized to it
  uint64_t select_batches = 0;    // batches that ran with the bounded output
  uint64_t select_exits = 0;      // returns to the compacting path (floors rose)
  uint64_t list_dma_copies = 0;   // long candidate lists DMA-copied instead of read in place
  uint64_t candidates = 0;        // above-threshold (bin, level, template) entries returned by the device
  uint64_t shared_series_batches = 0;  // batches that read another pipeline's series in place
  uint64_t peer_series_copies = 0;     // series taken device to device (peer / D2D), not from the host
};

class Backend {
 public:
  virtual ~Backend() = default;
  virtual const char* name() const = 0;
  // Per-WU setup: upload the series, whiten/zap it if opt.white (series is
  // updated in place with the whitened data).
  virtual int setup(const SearchGeometry& g, const SearchOptions& opt, std::vector<float>& series,
                    const std::vector<ZapRange>& zaps) = 0;
  // the same from the whole work unit (series = wu.samples): a device backend
  // may upload the stored payload and unpack it itself
  virtual int setup_wu(const SearchGeometry& g, const SearchOptions& opt, WorkUnit& wu,
                       const std::vector<ZapRange>& zaps) {
    return setup(g, opt, wu.samples, zaps);
  }
  // Process n templates with device thresholds thr (<= the sequential
  // thresholds of every template in the batch).
  virtual int process(const TemplateInput* t, int n, const float thr[kNumHarmonicLevels],
                      std::vector<TemplateCands>& out) = 0;
  // Take `first`'s prepared (whitened) series without a host round trip (same
  // device: read in place; another device: peer copy). can_setup_from() is
  // decided before `first` is set up; setup_from() == -1: not applicable,
  // > 0: an error code of the backend (e.g. a device allocation failure).
  virtual bool can_setup_from(const Backend& first, const SearchGeometry& g) const {
    (void)first;
    (void)g;
    return false;
  }
  virtual int setup_from(const Backend& first, const SearchGeometry& g) {
    (void)first;
    (void)g;
    return -1;
  }
  // Debug dumps (-z): the prepared series this backend searches and one
  // template's normalised power spectrum (fft_size bins). -1: not available.
  virtual int debug_buffers(const TemplateInput& t, std::vector<float>& series, std::vector<float>& ps) {
    (void)t;
    (void)series;
    (void)ps;
    return -1;
  }
  virtual int preferred_batch() const = 0;
  virtual int device() const { return -1; }
  // one-time start-up costs of the backend's first work, callable on another
  // thread before setup (HIP: code objects, copy kernels); 0 on success
  virtual int warm_up() { return 0; }
  virtual BackendStats stats() const { return {}; }
  // Pipelined form of process(): up to max_in_flight() batches submitted
  // before the oldest is completed; complete() returns results in submission
  // order. The default queues the arguments and runs process() inside
  // complete() (the HIP backend launches at submit()).
  virtual int max_in_flight() const { return 1; }
  virtual int submit(const TemplateInput* t, int n, const float thr[kNumHarmonicLevels]) {
    Pending p;
    p.t = t;
    p.n = n;
    for (int h = 0; h < kNumHarmonicLevels; ++h) p.thr[h] = thr[h];
    pending_.push_back(p);
    return 0;
  }
  virtual int complete(std::vector<TemplateCands>& out) {
    if (pending_.empty()) return -1;
    const Pending p = pending_.front();
    pending_.pop_front();
    return process(p.t, p.n, p.thr, out);
  }

 private:
  struct Pending {
    const TemplateInput* t;
    int n;
    float thr[kNumHarmonicLevels];
  };
  std::deque<Pending> pending_;
};

std::unique_ptr<Backend> make_cpu_backend();
// no-compute backend returning synthetic candidate lists (applier load tests)
std::unique_ptr<Backend> make_replay_backend(int per_level, int batch);
// device < 0: auto (BOINC gpu_device_num / first device)
// True when the HIP pipeline has an FFT plan for this geometry: the three-pass
// FFT for N/2 = L1*L2*L3 over the compiled lengths (fft_passes.hip), else the
// chirp-z transform over such a length (bluestein_kernels.hpp; every N up to
// 2^31 / 2).
bool hip_backend_supports(const SearchGeometry& g);
std::unique_ptr<Backend> make_hip_backend(int device, int batch, int* err);
// Start the HIP runtime (device enumeration; no context is created, so the
// blocking-sync flag can still be set): called on a helper thread while the
// host reads the work unit, bank and zaplist.
void hip_runtime_warm_up();
// Host-side FFT twiddle tables of the geometry's plan, computed ahead (they are
// cached per plan and shared by every pipeline); meant to overlap the HIP
// runtime start-up.
void hip_prepare_host_tables(const SearchGeometry& g);
// Host waits on HIP work sleep (hipDeviceScheduleBlockingSync) instead of
// spinning; set before the first backend is created (the BOINC app does).
void hip_set_blocking_sync(bool on);
// Page-lock an existing host range for direct DMA (hipHostRegister) for the
// lifetime of the returned handle; empty handle if the runtime refuses.
std::shared_ptr<void> hip_pin_host(void* p, size_t bytes);
// Device running median (whitening kernel) for tests and timing: out has
// in.size() - W + 1 entries; `reps` timed launches after one warm-up.
int hip_running_median(int device, const std::vector<float>& in, uint32_t W, std::vector<float>& out, int reps,
                       double* ms_per_call);

}  // namespace brp
