#include "search.hpp"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <deque>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <thread>

#include "../boinc/runtime.hpp"
#include "../boinc/ipc.hpp"
#include "../core/errors.hpp"
#include "../core/fault.hpp"
#include "../core/trace.hpp"
#include "../core/io.hpp"
#include "../core/log.hpp"
#include "../core/stats.hpp"
#include "../core/cpu_backend.hpp"

#ifndef BRP_GIT_ID
#define BRP_GIT_ID "unknown"
#endif

namespace brp {

namespace {

double now_s() {
  using namespace std::chrono;
  return duration<double>(steady_clock::now().time_since_epoch()).count();
}

}  // namespace

// RA/DEC (hhmmss.s / ddmmss.s) to radians for the screensaver (demod_binary.c:745-771)
void sky_position(const DDHeader& h, SearchInfo& info) {
  float hrs = std::floor(h.RA / 10000.0);
  float min = std::floor((h.RA - 10000.0 * hrs) / 100.0);
  float sec = h.RA - 10000.0 * hrs - 100.0 * min;
  info.skypos_rac = M_PI * (hrs / 12.0 + min / 720.0 + sec / 43200.0);
  if (h.DEC < 0.0) {
    hrs = std::floor(-h.DEC / 10000.0);
    min = std::floor(-(h.DEC + 10000.0 * hrs) / 100.0);
    sec = -(h.DEC + 10000.0 * hrs + 100.0 * min);
    info.skypos_dec = -M_PI * (hrs / 180.0 + min / 10800.0 + sec / 648000.0);
  } else {
    hrs = std::floor(h.DEC / 10000.0);
    min = std::floor((h.DEC - 10000.0 * hrs) / 100.0);
    sec = h.DEC - 10000.0 * hrs - 100.0 * min;
    info.skypos_dec = M_PI * (hrs / 180.0 + min / 10800.0 + sec / 648000.0);
  }
  info.dispersion_measure = h.DM;
}

namespace {

void log_header(const DDHeader& h) {
  log_message(LOG_INFO, true, "Header contents:\n");
  log_message(LOG_INFO, false, "Original WAPP file: %s\n", h.originalfile);
  log_message(LOG_INFO, false, "Sample time in microseconds: %g\n", h.tsample);
  log_message(LOG_INFO, false, "Observation time in seconds: %.8g\n", h.tobs);
  log_message(LOG_INFO, false, "Time stamp (MJD): %.17g\n", h.timestamp);
  log_message(LOG_INFO, false, "Number of samples/record: %d\n", h.smprec);
  log_message(LOG_INFO, false, "Center freq in MHz: %.10g\n", h.fcenter);
  log_message(LOG_INFO, false, "Channel band in MHz: %.9g\n", h.fchan);
  log_message(LOG_INFO, false, "Number of channels/record: %d\n", h.nchan);
  log_message(LOG_INFO, false, "Nifs: %d\n", h.nifs);
  log_message(LOG_INFO, false, "RA (J2000): %.12g\n", h.RA);
  log_message(LOG_INFO, false, "DEC (J2000): %.12g\n", h.DEC);
  log_message(LOG_INFO, false, "Galactic l: %.7g\n", h.gal_l);
  log_message(LOG_INFO, false, "Galactic b: %.7g\n", h.gal_b);
  log_message(LOG_INFO, false, "Name: %s\n", h.name);
  log_message(LOG_INFO, false, "Lagformat: %d\n", h.lagformat);
  log_message(LOG_INFO, false, "Sum: %d\n", h.sum);
  log_message(LOG_INFO, false, "Level: %d\n", h.level);
  log_message(LOG_INFO, false, "AZ at start: %.9g\n", h.AZstart);
  log_message(LOG_INFO, false, "ZA at start: %.9g\n", h.ZAstart);
  log_message(LOG_INFO, false, "AST at start: %.9g\n", h.ASTstart);
  log_message(LOG_INFO, false, "LST at start: %.9g\n", h.LSTstart);
  log_message(LOG_INFO, false, "Project ID: %s\n", h.proj_id);
  log_message(LOG_INFO, false, "Observers: %s\n", h.observers);
  log_message(LOG_INFO, false, "File size (bytes): %d\n", h.filesize);
  log_message(LOG_INFO, false, "Data size (bytes): %d\n", h.datasize);
  log_message(LOG_INFO, false, "Number of samples: %d\n", h.nsamples);
  log_message(LOG_INFO, false, "Trial dispersion measure: %g cm^-3 pc\n", h.DM);
  log_message(LOG_INFO, false, "Scale factor: %g\n", h.scale);
}

// Results of one dispatched batch, applied in template order by the driver.
struct BatchResult {
  uint32_t first = 0;
  int rc = 0;
  std::vector<TemplateCands> cands;
};

}  // namespace

int finalize_output(const SearchOptions& opt, const SearchGeometry& g, uint32_t n_done, CandidateTable& table,
                    const std::string& exec_name) {
  if (!opt.checkpointfile.empty()) {
    Checkpoint cp;
    std::memset(&cp.header, 0, sizeof(cp.header));
    cp.header.n_template = n_done;
    std::snprintf(cp.header.originalfile, sizeof(cp.header.originalfile), "%s", opt.inputfile.c_str());
    std::memcpy(cp.cands, table.data(), sizeof(cp.cands));
    int rc = write_checkpoint(opt.checkpointfile, cp);
    if (rc) return rc;
  }
  if (opt.outputfile.empty()) return 0;
  ResultHeaderInfo info;
  info.write_header = std::getenv("BRP_NO_RESULT_HEADER") == nullptr;
  const boinc::InitData& id = boinc::init_data();
  if (id.valid) {
    info.user_id = id.userid;
    info.user_name = id.user_name;
    info.host_id = id.hostid;
    info.host_cpid = id.host_cpid;
  } else if (info.write_header) {
    log_message(LOG_WARN, true, "User/host details unavailable...\n");
  }
  std::string ex = exec_name;
  const size_t slash = ex.find_last_of("\\/");
  if (slash != std::string::npos) ex = ex.substr(slash + 1);
  info.exec_name = ex;
  info.git_id = BRP_GIT_ID;
  info.boinc_rev = boinc::is_standalone() ? "standalone" : "brp-app-runtime";
  CPCand cands[kCandTotal];
  std::memcpy(cands, table.data(), sizeof(cands));
  return write_results(opt.outputfile, cands, g.t_obs_d, info);
}


struct SearchSession::Impl {
  SearchOptions opt;
  SearchControl ctl;
  TemplateBank bank;
  WorkUnit wu;
  SearchGeometry g;
  SearchInfo info;
  std::vector<ZapRange> zaps;
  std::vector<TemplateInput> tin;
  std::vector<std::unique_ptr<Backend>> backends;
  std::vector<float> series;  // whitened (or raw) series used for templates
  std::shared_ptr<void> wu_pin;  // wu.samples page-locked for the per-pass upload (released first)
  // floors of the table being applied (published after every batch) and the
  // external (other ranks') floors; float bits in atomics
  std::atomic<uint32_t> own_floor[kNumHarmonicLevels] = {};
  std::atomic<uint32_t> ext_floor[kNumHarmonicLevels] = {};
  void publish_floors(const CandidateTable& t) {
    for (int h = 0; h < kNumHarmonicLevels; ++h) {
      const float f = static_cast<float>(t.floor_power(h));
      uint32_t b;
      std::memcpy(&b, &f, sizeof(b));
      own_floor[h].store(b, std::memory_order_relaxed);
    }
  }
  float ext(int h) const {
    const uint32_t b = ext_floor[h].load(std::memory_order_relaxed);
    float f;
    std::memcpy(&f, &b, sizeof(f));
    return f;
  }
};

void SearchSession::local_floors(float out[kNumHarmonicLevels]) const {
  for (int h = 0; h < kNumHarmonicLevels; ++h) {
    const uint32_t b = impl_->own_floor[h].load(std::memory_order_relaxed);
    std::memcpy(&out[h], &b, sizeof(float));
  }
}

void SearchSession::raise_external_floors(const float f[kNumHarmonicLevels]) {
  for (int h = 0; h < kNumHarmonicLevels; ++h) {
    // non-negative floats order like their bit patterns: an atomic max on the bits
    if (!(f[h] > 0.0f)) continue;
    uint32_t b;
    std::memcpy(&b, &f[h], sizeof(b));
    uint32_t cur = impl_->ext_floor[h].load(std::memory_order_relaxed);
    while (b > cur && !impl_->ext_floor[h].compare_exchange_weak(cur, b, std::memory_order_relaxed)) {
    }
  }
}

void SearchSession::reset_external_floors() {
  for (int h = 0; h < kNumHarmonicLevels; ++h) {
    impl_->ext_floor[h].store(0, std::memory_order_relaxed);
    impl_->own_floor[h].store(0, std::memory_order_relaxed);
  }
}

SearchSession::SearchSession() : impl_(new Impl) {}
SearchSession::~SearchSession() = default;
const SearchGeometry& SearchSession::geometry() const { return impl_->g; }
const TemplateBank& SearchSession::bank() const { return impl_->bank; }
const WorkUnit& SearchSession::work_unit() const { return impl_->wu; }
const SearchOptions& SearchSession::options() const { return impl_->opt; }
uint32_t SearchSession::total() const { return static_cast<uint32_t>(impl_->bank.size()); }

BackendStats SearchSession::stats() const {
  BackendStats t;
  for (auto& be : impl_->backends) {
    const BackendStats s = be->stats();
    t.busy_span_ms += s.busy_span_ms;
    t.whiten_ms += s.whiten_ms;
    t.templates += s.templates;
    t.batches += s.batches;
    t.overflow_reruns += s.overflow_reruns;
    t.tie_reruns += s.tie_reruns;
    t.select_batches += s.select_batches;
    t.select_exits += s.select_exits;
    t.list_dma_copies += s.list_dma_copies;
    t.candidates += s.candidates;
    t.shared_series_batches += s.shared_series_batches;
    t.peer_series_copies += s.peer_series_copies;
  }
  return t;
}

int SearchSession::open(const SearchOptions& opt, const SearchControl& ctl) {
  Impl& d = *impl_;
  d.opt = opt;
  d.ctl = ctl;
  trace::phase("open");
  // the HIP runtime starts (device enumeration) while the host reads the
  // bank, the work unit and the zaplist (whole-process wall time, the
  // reference benchmark's /usr/bin/time protocol)
  std::thread hip_start;
  if (!opt.use_cpu && std::getenv("BRP_REPLAY_BACKEND") == nullptr) hip_start = std::thread(hip_runtime_warm_up);
  struct Joiner {
    std::thread& t;
    ~Joiner() {
      if (t.joinable()) t.join();
    }
  } join_hip_start{hip_start};
  int rc = read_template_bank(opt.templatebank, d.bank);
  if (rc) return rc;
  trace::phase("bank read");
  log_message(LOG_DEBUG, true, "Total amount of templates: %zu\n", d.bank.size());
  d.tin.resize(d.bank.size());
  for (size_t t = 0; t < d.bank.size(); ++t)
    d.tin[t] = TemplateInput{static_cast<float>(d.bank.P[t]), static_cast<float>(d.bank.tau[t]),
                             static_cast<float>(d.bank.Psi0[t])};
  rc = read_work_unit(opt.inputfile, d.wu);
  if (rc) return rc;
  trace::phase("work unit read");
  if (opt.debug) log_header(d.wu.header);
  sky_position(d.wu.header, d.info);
  rc = derive_geometry(d.wu.header, opt, d.g);
  if (rc) return rc;
  if (opt.white) {
    if (opt.zaplistfile.empty()) {
      log_message(LOG_ERROR, true, "Whitening requested but no zaplist file given (-l).\n");
      return RADPUL_EFILE;
    }
    rc = read_zaplist(opt.zaplistfile, d.zaps);
    if (rc) return rc;
  }
  if (opt.debug) {
    log_message(LOG_INFO, true, "Derived global search parameters:\n");
    log_message(LOG_INFO, false, "f_A probability = %g\n", opt.fA);
    log_message(LOG_INFO, false, "single bin prob(P_noise > P_thr) = %g\n", d.g.prob);
    const char* names[5] = {"thr1", "thr2", "thr4", "thr8", "thr16"};
    for (int h = 0; h < 5; ++h)
      log_message(LOG_INFO, false, "%s = %g\n", names[h], 0.5 * chisq_Qinv_even(d.g.prob, 1 << h));
  }
  if (hip_start.joinable()) {
    hip_prepare_host_tables(d.g);  // host work while the runtime starts
    trace::phase("host FFT tables");
    hip_start.join();
  }
  trace::phase("HIP runtime up");
  // one backend per device; with the CPU golden model, one per worker thread
  int ngpu = std::max(1, ctl.gpus);
  if (const char* rep = std::getenv("BRP_REPLAY_BACKEND")) {
    // applier load test: ctl.gpus x ctl.pipelines no-compute backends
    const int nb = ngpu * std::max(1, ctl.pipelines);
    for (int k = 0; k < nb; ++k) d.backends.push_back(make_replay_backend(std::atoi(rep), std::max(1, opt.batch)));
    return 0;
  }
  if (!d.opt.use_cpu && !hip_backend_supports(d.g)) {
    // Every N the reference can form on a real work unit has a plan: the
    // three-pass FFT for N/2 = L1*L2*L3 over 16*2^a*3^b*5^c*7^d lengths, the chirp-z
    // transform over such a length for all others (convolution length < 2^31,
    // i.e. N < ~2^30). Beyond that the product path refuses loudly; it never
    // switches to the CPU golden model behind the user's back.
    log_message(LOG_ERROR, true, "No HIP FFT plan for N = %u (padding %.3f).\n", d.g.nsamples, d.opt.padding);
    return RADPUL_HIP_FFT_PLAN;
  }
  // HIP: ctl.pipelines backends per device, consecutive backends on one device
  const int per_dev = d.opt.use_cpu ? 1 : std::max(1, ctl.pipelines);
  const int nback = ngpu * per_dev;
  boinc::begin_critical_section();
  // each device's first pipeline warms up (code objects, the runtime's copy
  // kernels) on a thread while the device's other pipelines create their
  // streams: ~25 ms of one-time cost off the critical path (round 6,
  // profiles/app_phases_r6.txt); BRP_WARM_UP=0: in line with the first work
  static const bool warm = std::getenv("BRP_WARM_UP") == nullptr || std::atoi(std::getenv("BRP_WARM_UP")) != 0;
  std::vector<std::thread> warmers;
  struct WarmJoiner {
    std::vector<std::thread>& w;
    ~WarmJoiner() {
      for (auto& t : w)
        if (t.joinable()) t.join();
    }
  } join_warmers{warmers};
  for (int kb = 0; kb < nback; ++kb) {
    const int k = kb / per_dev;  // device index
    std::unique_ptr<Backend> b;
    if (d.opt.use_cpu) {
      b = make_cpu_backend();
    } else {
      int dev = opt.device;
      if (!ctl.devices.empty()) dev = ctl.devices[kb % ctl.devices.size()];
      else if (ngpu > 1) dev = k;
      else if (dev < 0 && boinc::init_data().gpu_device_num >= 0) dev = boinc::init_data().gpu_device_num;
      int err = 0;
      b = make_hip_backend(dev, opt.batch, &err);
      if (!b) {
        boinc::end_critical_section();
        return err ? err : RADPUL_HIP_DEVICE_FIND;
      }
    }
    d.backends.push_back(std::move(b));
    if (warm && !d.opt.use_cpu && kb % per_dev == 0 && per_dev > 1) {
      Backend* first = d.backends.back().get();
      warmers.emplace_back([first] {
        if (const int rc = first->warm_up()) log_message(LOG_DEBUG, true, "Backend warm-up failed (%d).\n", rc);
      });
    }
  }
  for (auto& t : warmers) t.join();
  boinc::end_critical_section();
  trace::phase("backends created");
  return 0;
}

int SearchSession::prepare() {
  Impl& d = *impl_;
  trace::Range range("brp:prepare");
  boinc::begin_critical_section();
  // every other backend takes the first one's whitened series device to
  // device (same device: in place; other devices: peer copy from that
  // device's first pipeline, which copied it from backend 0 over xGMI), so
  // the host copy-back of the whitened series is only needed otherwise
  const size_t nb = d.backends.size();
  std::vector<size_t> src(nb, 0);
  for (size_t k = 1; k < nb; ++k) {
    const int dev = d.backends[k]->device();
    for (size_t j = 0; j < k; ++j)
      if (dev >= 0 && d.backends[j]->device() == dev) {
        src[k] = j;
        break;
      }
  }
  bool device_all = true;
  for (size_t k = 1; k < nb; ++k) device_all = device_all && d.backends[k]->can_setup_from(*d.backends[src[k]], d.g);
  SearchOptions opt0 = d.opt;
  opt0.device_series = device_all;
  const bool hip0 = std::strcmp(d.backends[0]->name(), "hip") == 0;
  if (hip0 && !d.wu_pin && !d.wu.packed.empty())  // the payload is what crosses PCIe (setup_wu)
    d.wu_pin = hip_pin_host(d.wu.packed.data(), d.wu.packed.size());
  // a HIP backend that keeps the whitened series on the device only reads
  // the raw samples: upload them straight from the (page-locked) WU buffer
  const bool direct = hip0 && device_all;
  if (!direct) d.series = d.wu.samples;
  int rc = direct ? d.backends[0]->setup_wu(d.g, opt0, d.wu, d.zaps) : d.backends[0]->setup(d.g, opt0, d.series, d.zaps);
  if (rc) {
    boinc::end_critical_section();
    return rc;
  }
  trace::phase("pipeline 0 set up + whitened");
  SearchOptions opt_nw = d.opt;
  opt_nw.white = false;
  opt_nw.prewhitened = d.opt.white;
  for (size_t k = 1; k < nb; ++k) {
    rc = d.backends[k]->setup_from(*d.backends[src[k]], d.g);
    if (rc == 0) continue;
    if (rc > 0) {  // e.g. RADPUL_HIP_MEM_ALLOC_DEVICE: the wrapper's temporary exit
      boinc::end_critical_section();
      return rc;
    }
    if (device_all) {
      // the host never received the whitened series
      log_message(LOG_ERROR, true, "Pipeline %zu could not take the whitened series from pipeline %zu.\n", k, src[k]);
      boinc::end_critical_section();
      return RADPUL_HIP_MEM_COPY_HOST_DEVICE;
    }
    std::vector<float> s = d.series;
    rc = d.backends[k]->setup(d.g, opt_nw, s, d.zaps);
    if (rc) {
      boinc::end_critical_section();
      return rc;
    }
  }
  boinc::end_critical_section();
  trace::phase("pipelines set up");
  if (d.opt.debug && !d.opt.dump_dir.empty() && !d.tin.empty()) return dump_debug_buffers();
  return 0;
}

// -z with a dump directory: the searched (whitened) series, template 0's
// resampled series and its power spectrum as text, one value per line
// (reference dumpFloatBufferToTextFile, erp_utilities.cpp:216-233, and the
// device-buffer variant cuda_utilities.c:283-320). The resampled series comes
// from the host model: the device gather uses the same nearest indices bit for
// bit but never materialises the series (it is fused into FFT pass 1).
int SearchSession::dump_debug_buffers() {
  Impl& d = *impl_;
  std::vector<float> series, ps, x;
  boinc::begin_critical_section();
  int rc = d.backends[0]->debug_buffers(d.tin[0], series, ps);
  boinc::end_critical_section();
  if (rc) {
    log_message(LOG_WARN, true, "Debug buffers not available from the %s backend.\n", d.backends[0]->name());
    return 0;
  }
  const TemplateInput& t = d.tin[0];
  const ResampParams p = make_resamp_params(d.g.nsamples, d.g.n_unpadded, d.g.fft_size, d.g.dt, d.g.step_inv, t.P,
                                            t.tau, t.Psi0);
  cpu_resample(series.data(), p, x, nullptr, nullptr);
  const std::string dir = d.opt.dump_dir + "/";
  if ((rc = dump_float_buffer(series.data(), series.size(), dir + "dump_series.txt"))) return rc;
  if ((rc = dump_float_buffer(x.data(), x.size(), dir + "dump_resampled_t0.txt"))) return rc;
  return dump_float_buffer(ps.data(), ps.size(), dir + "dump_power_t0.txt");
}

int SearchSession::run(uint32_t begin, uint32_t end, CandidateTable& table, SearchResult& res,
                       const TemplateHook& hook) {
  Impl& d = *impl_;
  trace::Range range("brp:templates");
  const SearchGeometry& g = d.g;
  end = std::min<uint32_t>(end, total());
  if (begin >= end) return 0;
  const int B = std::max(1, d.backends[0]->preferred_batch());

  // Batches are dealt to the devices; results are applied in template order so
  // the table evolves exactly as in the sequential reference loop
  // (demod_binary.c:1180-1443). Device thresholds lag by at most the batches in
  // flight, which only adds bins that the in-order application rejects.
  std::mutex mu;
  std::condition_variable cv;
  std::map<uint32_t, BatchResult> ready;
  float thr_shared[kNumHarmonicLevels];
  table.thresholds(g.chi2_thr, thr_shared);
  d.publish_floors(table);
  std::atomic<uint32_t> next_first{begin};
  std::atomic<bool> stop{false};
  // Batch sizes shrink over the last templates of the range (below two
  // batches per in-flight slot of all pipelines) so that the pipelines finish
  // together: a shard's tail then idles the GPU for about one template instead
  // of one full batch (serial launch groups make batches 4 templates long).
  int slots_all = 0;
  for (auto& be : d.backends) slots_all += std::max(1, be->max_in_flight());
  const uint32_t tail = 2u * static_cast<uint32_t>(std::max(1, slots_all)) * static_cast<uint32_t>(B);
  auto take = [&](uint32_t& first) -> int {
    uint32_t f = next_first.load(std::memory_order_relaxed);
    if (f < end && end - f > tail + static_cast<uint32_t>(B)) {
      // far from the tail: one fetch_add (a CAS loop contends when many
      // pipelines take batches at once); one landing in the tail is still exact
      f = next_first.fetch_add(static_cast<uint32_t>(B));
      if (f >= end) return 0;
      first = f;
      return static_cast<int>(std::min<uint32_t>(static_cast<uint32_t>(B), end - f));
    }
    for (;;) {
      if (f >= end) return 0;
      const uint32_t rem = end - f;
      const uint32_t n = std::min<uint32_t>(
          std::min<uint32_t>(static_cast<uint32_t>(B), rem),
          std::max<uint32_t>(1u, rem / static_cast<uint32_t>(2 * std::max(1, slots_all))));
      if (next_first.compare_exchange_weak(f, f + n)) {
        first = f;
        return static_cast<int>(n);
      }
    }
  };
  // Each worker keeps up to max_in_flight() batches of its backend submitted
  // (the next batch is launched while the previous one runs), completing them
  // in submission order.
  auto worker = [&](Backend* be) {
    const int depth = std::max(1, be->max_in_flight());
    std::deque<uint32_t> inflight;  // first template of each submitted batch
    auto publish = [&](BatchResult&& br) {
      {
        std::lock_guard<std::mutex> lk(mu);
        ready.emplace(br.first, std::move(br));
      }
      cv.notify_all();
    };
    for (;;) {
      while (static_cast<int>(inflight.size()) < depth) {
        // a suspended task starts no GPU work; batches already launched
        // finish inside their critical section (demod_binary.c:1241-1296)
        boinc::suspend_point();
        if (stop.load()) break;
        uint32_t first = 0;
        const int n = take(first);
        if (n == 0) break;
        float thr[kNumHarmonicLevels];
        {
          std::lock_guard<std::mutex> lk(mu);
          std::memcpy(thr, thr_shared, sizeof(thr));
        }
        // Other ranks' floors prune the device output: a bin below every
        // merged-table floor can never enter it. The device emits p > thr, so
        // the threshold is the float just below the external floor: a bin whose
        // power equals it is still emitted, and the in-order tie rules
        // (demod_binary.c:1345, strict >) decide it exactly as in the merge.
        for (int h = 0; h < kNumHarmonicLevels; ++h) {
          const float e = d.ext(h);
          if (e > 0.0f) thr[h] = std::fmax(thr[h], std::nextafter(e, 0.0f));
        }
        boinc::begin_critical_section();
        const int rc = be->submit(&d.tin[first], n, thr);
        if (rc) {
          boinc::end_critical_section();
          BatchResult br;
          br.first = first;
          br.rc = rc;
          publish(std::move(br));
          continue;
        }
        inflight.push_back(first);
      }
      if (inflight.empty()) return;
      BatchResult br;
      br.first = inflight.front();
      inflight.pop_front();
      br.rc = be->complete(br.cands);
      boinc::end_critical_section();
      publish(std::move(br));
    }
  };
  std::vector<std::thread> threads;
  for (auto& be : d.backends) threads.emplace_back(worker, be.get());

  uint32_t applied = begin;
  int rc = 0;
  bool quit = false;
  std::vector<uint32_t> pages;  // distinct dirty pages per level (statistics)
  SearchInfo& info = d.info;
  while (applied < end && !quit) {
    BatchResult br;
    {
      std::unique_lock<std::mutex> lk(mu);
      cv.wait(lk, [&] { return ready.count(applied) > 0; });
      br = std::move(ready[applied]);
      ready.erase(applied);
    }
    if (br.rc) {
      rc = br.rc;
      break;
    }
    for (size_t k = 0; k < br.cands.size() && !quit; ++k) {
      const uint32_t t = br.first + static_cast<uint32_t>(k);
      const TemplateInput& ti = d.tin[t];
      float thrA[kNumHarmonicLevels];
      table.thresholds(g.chi2_thr, thrA);
      unsigned char binned[kBinsScreensaver] = {0};
      for (int h = 0; h < kNumHarmonicLevels; ++h) {
        const std::vector<BinPower>& lv = br.cands[k].level[h];
        table.apply_level(h, lv.data(), lv.size(), thrA[h], ti.P, ti.tau, ti.Psi0);
        if (lv.empty()) continue;
        pages.clear();
        for (const BinPower& bp : lv)
          if (bp.power > thrA[h]) pages.push_back(bp.bin >> kLogPsPageSize);
        std::sort(pages.begin(), pages.end());
        res.dirty_pages += static_cast<uint64_t>(std::unique(pages.begin(), pages.end()) - pages.begin());
        if (h == 2) {
          const float powerscale = 100.0f / 255.0f;
          const float stepscale = static_cast<float>(kBinsScreensaver) / static_cast<float>(g.fundamental_idx_hi);
          for (const BinPower& bp : lv) {
            const int bin_ss = static_cast<int>(stepscale * bp.bin);
            if (bin_ss >= 0 && bin_ss < kBinsScreensaver && bp.power > powerscale * binned[bin_ss])
              binned[bin_ss] = static_cast<unsigned char>(std::min(bp.power / powerscale, 255.0f));
          }
        }
      }
      info.orbital_radius = ti.tau;
      info.orbital_period = ti.P;
      info.orbital_phase = ti.Psi0;
      std::memcpy(info.power_spectrum, binned, sizeof(binned));
      ++res.templates_run;
      if (hook && !hook(t + 1, info)) quit = true;
    }
    applied = br.first + static_cast<uint32_t>(br.cands.size());
    {
      std::lock_guard<std::mutex> lk(mu);
      table.thresholds(g.chi2_thr, thr_shared);
    }
    d.publish_floors(table);
  }
  stop.store(true);
  for (auto& th : threads) th.join();
  if (quit) res.interrupted = true;
  return rc;
}

namespace {
std::atomic<bool> g_keep_device_state{false};
}  // namespace

void set_keep_device_state_on_return(bool on) { g_keep_device_state.store(on); }

int run_search(const SearchOptions& opt, const SearchControl& ctl, SearchResult& res) {
  const double t_start = now_s();
  res = SearchResult();
  log_message(LOG_INFO, true, "Starting data processing...\n");
  if (fault_enabled("resource_error")) return RADPUL_HIP_MEM_ALLOC_HOST;
  std::unique_ptr<SearchSession> owner(new SearchSession);
  struct Keep {
    std::unique_ptr<SearchSession>& s;
    ~Keep() {
      if (g_keep_device_state.load()) (void)s.release();  // left to process exit
    }
  } keep{owner};
  SearchSession& session = *owner;
  int rc = session.open(opt, ctl);
  if (rc) return rc;
  const uint32_t total = session.total();
  res.templates_total = total;
  res.geom = session.geometry();
  const SearchGeometry& g = res.geom;

  // checkpoint restore (demod_binary.c:546-652)
  CandidateTable& table = res.table;
  uint32_t counter = 0;
  if (ctl.use_checkpoint && !opt.checkpointfile.empty()) {
    Checkpoint cp;
    bool exists = false;
    rc = read_checkpoint(opt.checkpointfile, cp, exists);
    if (rc) return rc;
    if (!exists) {
      log_message(LOG_INFO, true, "Checkpoint file unavailable: %s.\n", opt.checkpointfile.c_str());
      log_message(LOG_INFO, false, "Starting from scratch...\n");
      if (opt.inputfile.size() >= static_cast<size_t>(kFnLength)) {
        log_message(LOG_ERROR, true, "Couldn't write input file %s name to checkpoint header.\n",
                    opt.inputfile.c_str());
        return RADPUL_EFILE;
      }
    } else {
      if (cp.header.n_template == total) {
        log_message(LOG_INFO, true, "Thank you but this work unit has already been processed completely...\n");
      } else if (cp.header.n_template < total) {
        log_message(LOG_INFO, true, "Continuing work on %s at template no. %u\n", cp.header.originalfile,
                    cp.header.n_template);
      } else {
        log_message(LOG_ERROR, true,
                    "Header checkpoint file %s contains inconsistent information about number of templates done "
                    "(%u > %u).\n",
                    opt.checkpointfile.c_str(), cp.header.n_template, total);
        return RADPUL_EFILE;
      }
      cp.header.originalfile[kFnLength - 1] = 0;
      if (opt.inputfile != cp.header.originalfile) {
        log_message(LOG_ERROR, true,
                    "Input file on command line %s doesn't agree with input file %s from checkpoint header.\n",
                    opt.inputfile.c_str(), cp.header.originalfile);
        return RADPUL_EFILE;
      }
      std::memcpy(table.data(), cp.cands, sizeof(cp.cands));
      counter = cp.header.n_template;
      if (opt.debug) {
        log_message(LOG_DEBUG, true, "Candidates found so far:\n");
        for (int i = 0; i < kCandTotal; ++i) {
          const CPCand& c = table.data()[i];
          log_message(LOG_DEBUG, false, "%u %6.12f %6.12f %6.12f %6.12f %u\n", c.f0, c.power, c.P_b, c.tau, c.Psi,
                      c.n_harm);
        }
      }
    }
  }
  const uint32_t begin = std::max(counter, ctl.begin);
  const uint32_t end = (ctl.end == 0 || ctl.end > total) ? total : ctl.end;
  if (begin < end) {
    rc = session.prepare();
    if (rc) return rc;
  }
  res.t_setup = now_s() - t_start;

  const double t_loop = now_s();
  long kill_after = -1, segv_after = -1;
  std::string fault_arg;
  if (fault_enabled("kill_after_template", &fault_arg)) kill_after = std::atol(fault_arg.c_str());
  if (fault_enabled("segv_after_template", &fault_arg)) segv_after = std::atol(fault_arg.c_str());
  long slow_ms = 0;
  if (fault_enabled("slow_template", &fault_arg)) slow_ms = std::atol(fault_arg.c_str());
  int cp_rc = 0;
  auto hook = [&](uint32_t done, const SearchInfo& info) -> bool {
    counter = done;
    if (ctl.progress_every <= 1 || counter % ctl.progress_every == 0) {
      if (ipc::update_due()) ipc::update_shmem(info);
      boinc::fraction_done((counter + 1.0) / total);
    }
    if (ctl.on_template) ctl.on_template(counter, total);
    if (ctl.use_checkpoint && !opt.checkpointfile.empty() && boinc::time_to_checkpoint()) {
      Checkpoint cp;
      std::memset(&cp.header, 0, sizeof(cp.header));
      cp.header.n_template = counter;
      std::snprintf(cp.header.originalfile, sizeof(cp.header.originalfile), "%s", opt.inputfile.c_str());
      std::memcpy(cp.cands, table.data(), sizeof(cp.cands));
      trace::Range range("brp:checkpoint");
      cp_rc = write_checkpoint(opt.checkpointfile, cp);
      if (cp_rc) {
        boinc::end_critical_section();
        return false;
      }
      log_message(LOG_INFO, true, "Checkpoint committed!\n");
      boinc::checkpoint_completed();
    }
    if (kill_after >= 0 && counter >= static_cast<uint32_t>(kill_after)) boinc::request_quit();
    if (segv_after >= 0 && counter >= static_cast<uint32_t>(segv_after)) {
      // a real invalid store (not raise()) so the crash report shows this frame
      static volatile uintptr_t no_page = 0;
      *reinterpret_cast<volatile int*>(no_page) = 1;
    }
    if (slow_ms > 0) std::this_thread::sleep_for(std::chrono::milliseconds(slow_ms));
    // template boundary: a suspended task waits here (no GPU work is queued)
    boinc::suspend_point();
    const boinc::Status st = boinc::get_status();
    return !(st.quit_request || st.abort_request || st.no_heartbeat);
  };
  rc = session.run(begin, end, table, res, hook);
  res.t_templates = now_s() - t_loop;
  trace::phase("templates done");
  res.templates_done = counter;
  res.stats = session.stats();
  if (rc) return rc;
  if (cp_rc) return cp_rc;
  if (res.interrupted) {
    // the reference exits without a final checkpoint (demod_binary.c:1489-1492)
    log_message(LOG_WARN, true, "BOINC wants us to quit prematurely or we lost contact! Exiting...\n");
    res.t_total = now_s() - t_start;
    return 0;
  }
  if (ctl.write_output) {
    log_message(LOG_DEBUG, true, "Search done!\n");
    trace::Range range("brp:finalize_output");
    rc = finalize_output(opt, g, counter, table, "einsteinbinary_mi355x");
    if (rc) return rc;
    trace::phase("output written");
  }
  log_message(LOG_INFO, true,
              "Statistics: count dirty SumSpec pages %llu (not checkpointed), Page Size %d, fundamental_idx_hi-window_2: %u\n",
              static_cast<unsigned long long>(res.dirty_pages), 1 << kLogPsPageSize,
              g.fundamental_idx_hi - g.window_2);
  res.t_total = now_s() - t_start;
  log_message(LOG_INFO, true, "Data processing finished successfully!\n");
  return 0;
}

}  // namespace brp
