#include "multi.hpp"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <thread>

#include "../boinc/runtime.hpp"
#include "../core/errors.hpp"
#include "../core/io.hpp"
#include "../core/log.hpp"
#include "../core/trace.hpp"
#include "../engine/hip_engine.hpp"

namespace brp {

namespace {

double now_s() {
  using namespace std::chrono;
  return duration<double>(steady_clock::now().time_since_epoch()).count();
}

bool same_shape(const SearchGeometry& a, const SearchGeometry& b) {
  return a.nsamples == b.nsamples && a.n_unpadded == b.n_unpadded && a.fft_size == b.fft_size &&
         a.window_2 == b.window_2 && a.fundamental_idx_hi == b.fundamental_idx_hi &&
         a.harmonic_idx_hi == b.harmonic_idx_hi && a.dt == b.dt && a.step_inv == b.step_inv;
}

// TB = B * batches in 64 bits, clamped to the bank rounded up to whole batches
uint32_t multi_block_templates_for(int B, uint32_t total, uint64_t batches) {
  const uint64_t b = static_cast<uint64_t>(std::max(1, B));
  const uint64_t cap = std::max<uint64_t>(b, (static_cast<uint64_t>(total) + b - 1) / b * b);
  return static_cast<uint32_t>(std::min<uint64_t>(b * std::max<uint64_t>(1, batches), cap));
}

}  // namespace

struct MultiSession::Impl {
  SearchOptions opt;
  SearchControl ctl;
  TemplateBank bank;
  std::vector<WorkUnit> wus;
  std::vector<SearchGeometry> geoms;
  std::vector<ZapRange> zaps;
  std::vector<std::unique_ptr<HipEngine>> engines;
  std::vector<std::string> inputs;
  uint32_t block_batches = 0;  // 0: BRP_MULTI_BLOCK / default
  bool shape_mismatch = false;
  SearchInfo info;
  std::vector<std::shared_ptr<void>> pins;  // page-locked WU sample buffers (direct uploads)
};

uint32_t multi_block_templates(int B, uint32_t total) {
  static const uint64_t env_batches = [] {
    const char* e = std::getenv("BRP_MULTI_BLOCK");
    return e ? static_cast<uint64_t>(std::max(1L, std::atol(e))) : 64ull;
  }();
  return multi_block_templates_for(B, total, env_batches);
}

MultiSession::MultiSession() : impl_(new Impl) {}
MultiSession::~MultiSession() = default;
size_t MultiSession::work_units() const { return impl_->wus.size(); }
uint32_t MultiSession::total() const { return static_cast<uint32_t>(impl_->bank.size()); }
const SearchGeometry& MultiSession::geometry() const { return impl_->geoms.at(0); }
void MultiSession::set_block_batches(uint32_t n) { impl_->block_batches = n; }
const SearchInfo& MultiSession::info() const { return impl_->info; }
bool MultiSession::shape_mismatch() const { return impl_->shape_mismatch; }

BackendStats MultiSession::stats() const {
  BackendStats t;
  for (auto& e : impl_->engines) {
    const BackendStats s = e->stats();
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

int MultiSession::open(const std::vector<std::string>& inputs, const SearchOptions& opt, const SearchControl& ctl) {
  Impl& d = *impl_;
  if (inputs.empty()) return RADPUL_EVAL;
  d.opt = opt;
  d.ctl = ctl;
  d.inputs = inputs;
  int rc = read_template_bank(opt.templatebank, d.bank);
  if (rc) return rc;
  if (opt.white) {
    if (opt.zaplistfile.empty()) {
      log_message(LOG_ERROR, true, "Whitening requested but no zaplist file given (-l).\n");
      return RADPUL_EFILE;
    }
    if ((rc = read_zaplist(opt.zaplistfile, d.zaps))) return rc;
  }
  d.wus.resize(inputs.size());
  d.geoms.resize(inputs.size());
  for (size_t k = 0; k < inputs.size(); ++k) {
    if ((rc = read_work_unit(inputs[k], d.wus[k]))) return rc;
    if ((rc = derive_geometry(d.wus[k].header, opt, d.geoms[k]))) return rc;
    if (!same_shape(d.geoms[k], d.geoms[0])) {
      log_message(LOG_WARN, true, "Work unit %s differs in shape from %s; batch only same-shape WUs.\n",
                  inputs[k].c_str(), inputs[0].c_str());
      d.shape_mismatch = true;
      return RADPUL_EVAL;
    }
  }
  sky_position(d.wus[0].header, d.info);
  if (!hip_backend_supports(d.geoms[0])) {
    log_message(LOG_ERROR, true, "No HIP FFT plan for N = %u.\n", d.geoms[0].nsamples);
    return RADPUL_HIP_FFT_PLAN;
  }
  const int np = std::max(1, ctl.gpus);
  for (int e = 0; e < np; ++e) {
    auto eng = std::make_unique<HipEngine>();
    int dev = opt.device;
    if (!ctl.devices.empty()) dev = ctl.devices[e % ctl.devices.size()];
    else if (np > 1) dev = e;
    if ((rc = eng->init(dev, opt.batch > 0 ? opt.batch : 8))) return rc;
    if ((rc = eng->set_slots(static_cast<uint32_t>(inputs.size())))) return rc;
    if (opt.ps_fp16 && !opt.white) {
      log_message(LOG_ERROR, true, "The fp16 power spectrum needs whitening (-W).\n");
      return RADPUL_EVAL;
    }
    eng->set_ps_fp16(opt.ps_fp16);
    d.engines.push_back(std::move(eng));
  }
  return 0;
}

int MultiSession::prepare() {
  Impl& d = *impl_;
  trace::Range range("brp:multi_prepare");
  const SearchGeometry& g = d.geoms[0];
  int rc;
  std::vector<std::vector<float>> prepared(d.wus.size());
  std::vector<float> mu0(d.wus.size(), 0.0f);
  bool all_same_device = true;
  for (auto& e : d.engines) all_same_device = all_same_device && e->device() == d.engines[0]->device();
  HipEngine& e0 = *d.engines[0];
  for (size_t k = 0; k < d.wus.size(); ++k) {
    // Whitening on one device only reads the raw samples (uploaded straight
    // from the page-locked WU buffer) and resets the padding offset to 0, so
    // neither a host copy nor the 4M-sample mean is needed then; otherwise the
    // (whitened) host copy feeds the engines on other devices.
    const bool direct = d.opt.white && all_same_device;
    if (!direct) prepared[k] = d.wus[k].samples;
    std::vector<float>& s = direct ? d.wus[k].samples : prepared[k];
    if (direct && d.pins.size() < d.wus.size()) d.pins.resize(d.wus.size());
    if (direct && !d.pins[k]) d.pins[k] = hip_pin_host(s.data(), s.size() * sizeof(float));
    double mean = 0.0;
    if (!d.opt.white) {
      for (float v : s) mean += v;
      mean = s.empty() ? 0.0 : mean / s.size();
    }
    if (k == 0) rc = e0.setup(g, s, static_cast<float>(mean));
    else rc = e0.load_slot(static_cast<uint32_t>(k), s, static_cast<float>(mean));
    if (rc) return rc;
    mu0[k] = static_cast<float>(mean);
    if (d.opt.white) {
      // per-WU geometry carries the WU's own t_obs for the zap bins; the
      // host copy of the whitened series is needed only by engines on
      // other devices
      if ((rc = e0.whiten(d.opt, d.zaps, s, static_cast<uint32_t>(k), !all_same_device))) return rc;
      mu0[k] = 0.0f;
    }
  }
  for (size_t e = 1; e < d.engines.size(); ++e) {
    HipEngine& en = *d.engines[e];
    if (en.device() == e0.device()) {
      // Pipelines on engine 0's device read its K whitened series in place
      // (like the single-WU session's adopt_series): one copy of each series
      // in the Infinity Cache instead of one per pipeline, and no uploads.
      // The first pass allocates this engine's buffers once.
      if (!en.ready_for(g) && (rc = en.setup(g, d.wus[0].samples, 0.0f))) return rc;
      if ((rc = en.adopt_series(e0)) == 0) continue;
      log_message(LOG_ERROR, true, "Pipeline %zu could not read pipeline 0's series in place.\n", e);
      return rc;
    }
    for (size_t k = 0; k < d.wus.size(); ++k) {
      if (k == 0) rc = en.setup(g, prepared[0], mu0[0]);
      else rc = en.load_slot(static_cast<uint32_t>(k), prepared[k], mu0[k]);
      if (rc) return rc;
    }
  }
  return 0;
}

int MultiSession::run(uint32_t begin, uint32_t end, std::vector<CandidateTable>& tables, MultiResult& res) {
  return run(std::vector<uint32_t>(impl_->wus.size(), begin), end, tables, res, MultiHook());
}

int MultiSession::run(const std::vector<uint32_t>& begins, uint32_t end, std::vector<CandidateTable>& tables,
                      MultiResult& res, const MultiHook& hook) {
  Impl& d = *impl_;
  trace::Range range("brp:multi_templates");
  const SearchGeometry& g = d.geoms[0];
  const uint32_t K = static_cast<uint32_t>(d.wus.size());
  if (begins.size() != K) return RADPUL_EVAL;
  end = std::min<uint32_t>(end == 0 ? total() : end, total());
  tables.resize(K);
  const uint32_t begin = *std::min_element(begins.begin(), begins.end());
  if (begin >= end) return 0;
  const double t0 = now_s();
  const int B = d.engines[0]->batch();
  // device thresholds per WU (lag by the batches in flight; exact ones on the host)
  std::vector<float> thr_wu(static_cast<size_t>(K) * kNumHarmonicLevels);
  for (uint32_t w = 0; w < K; ++w) tables[w].thresholds(g.chi2_thr, &thr_wu[w * kNumHarmonicLevels]);
  struct Batch {
    uint64_t first = 0;
    int rc = 0;
    std::vector<TemplateInput> tin;
    std::vector<TemplateCands> cands;
  };
  std::mutex mu;
  std::condition_variable cv;
  std::map<uint64_t, Batch> ready;
  std::atomic<uint64_t> next{0};
  std::atomic<bool> stop{false};
  // deal order: blocks of TB templates (a multiple of B), WU by WU within a
  // block. A batch then holds templates of one WU, and every WU still sees its
  // templates in increasing order. Long blocks keep all pipelines on the same
  // WU, so one 16 MB series (not K of them) competes with the pipelines' FFT
  // buffers for the 256 MB Infinity Cache. BRP_MULTI_BLOCK = batches per block.
  const uint32_t TB = d.block_batches ? multi_block_templates_for(B, end - begin, d.block_batches)
                                       : multi_block_templates(B, end - begin);
  std::vector<std::pair<uint32_t, uint32_t>> order;  // (template, WU)
  // deal blocks: end index in `order` and the template prefix complete after it
  std::vector<std::pair<uint64_t, uint32_t>> blocks;
  for (uint64_t t0 = begin; t0 < end; t0 += TB) {
    const uint32_t t_hi = static_cast<uint32_t>(std::min<uint64_t>(t0 + TB, end));
    for (uint32_t w = 0; w < K; ++w)
      for (uint32_t t = std::max<uint32_t>(static_cast<uint32_t>(t0), begins[w]); t < t_hi; ++t) order.emplace_back(t, w);
    blocks.emplace_back(order.size(), t_hi);
  }
  const uint64_t npairs = order.size();
  if (npairs == 0) return 0;
  // batches never cross a deal block: when the WUs resume from different
  // templates a block is not a multiple of B pairs, and a batch spanning two
  // blocks would put templates past the block's checkpoint prefix into the
  // tables that checkpoint describes
  std::vector<uint64_t> bstart;
  {
    uint64_t q = 0;
    for (const auto& blk : blocks) {
      for (; q < blk.first; q += static_cast<uint64_t>(B)) bstart.push_back(q);
      q = blk.first;
    }
    bstart.push_back(npairs);
  }
  const uint64_t nbatches = bstart.size() - 1;
  auto pair_input = [&](uint64_t q) {
    const uint32_t t = order[q].first;
    const uint32_t w = order[q].second;
    TemplateInput ti{static_cast<float>(d.bank.P[t]), static_cast<float>(d.bank.tau[t]),
                     static_cast<float>(d.bank.Psi0[t])};
    ti.wu = w;
    return ti;
  };
  // up to max_in_flight() batches submitted per engine (the next launched while
  // the previous runs), completed in submission order
  auto worker = [&](HipEngine* eng) {
    const int depth = std::max(1, eng->max_in_flight());
    std::deque<Batch> inflight;
    std::vector<float> thr;
    auto publish = [&](Batch&& bt) {
      {
        std::lock_guard<std::mutex> lk(mu);
        const uint64_t f = bt.first;
        ready.emplace(f, std::move(bt));
      }
      cv.notify_all();
    };
    for (;;) {
      while (static_cast<int>(inflight.size()) < depth) {
        boinc::suspend_point();  // no GPU work starts while the client has the task suspended
        if (stop.load()) break;
        const uint64_t bi = next.fetch_add(1);
        if (bi >= nbatches) break;
        const uint64_t first = bstart[bi];
        const int n = static_cast<int>(bstart[bi + 1] - first);
        Batch bt;
        bt.first = first;
        thr.assign(static_cast<size_t>(n) * kNumHarmonicLevels, 0.0f);
        for (int i = 0; i < n; ++i) bt.tin.push_back(pair_input(first + i));
        {
          std::lock_guard<std::mutex> lk(mu);
          for (int i = 0; i < n; ++i)
            std::memcpy(&thr[static_cast<size_t>(i) * kNumHarmonicLevels],
                        &thr_wu[static_cast<size_t>(bt.tin[i].wu) * kNumHarmonicLevels],
                        sizeof(float) * kNumHarmonicLevels);
        }
        boinc::begin_critical_section();
        bt.rc = eng->submit(bt.tin.data(), n, thr.data(), kNumHarmonicLevels);  // copies its inputs
        if (bt.rc) {
          boinc::end_critical_section();
          publish(std::move(bt));
          continue;
        }
        inflight.push_back(std::move(bt));
      }
      if (inflight.empty()) return;
      Batch bt = std::move(inflight.front());
      inflight.pop_front();
      bt.rc = eng->complete(bt.cands);
      boinc::end_critical_section();
      publish(std::move(bt));
    }
  };
  std::vector<std::thread> threads;
  for (auto& e : d.engines) threads.emplace_back(worker, e.get());
  uint64_t applied = 0;
  size_t next_block = 0;
  int rc = 0;
  while (applied < npairs) {
    Batch bt;
    {
      std::unique_lock<std::mutex> lk(mu);
      cv.wait(lk, [&] { return ready.count(applied) > 0; });
      bt = std::move(ready[applied]);
      ready.erase(applied);
    }
    if (bt.rc) {
      rc = bt.rc;
      break;
    }
    for (size_t i = 0; i < bt.cands.size(); ++i) {
      const TemplateInput& ti = bt.tin[i];
      CandidateTable& tab = tables[ti.wu];
      float thrA[kNumHarmonicLevels];
      tab.thresholds(d.geoms[ti.wu].chi2_thr, thrA);
      for (int h = 0; h < kNumHarmonicLevels; ++h) {
        const std::vector<BinPower>& lv = bt.cands[i].level[h];
        tab.apply_level(h, lv.data(), lv.size(), thrA[h], ti.P, ti.tau, ti.Psi0);
      }
      ++res.pairs_run;
    }
    applied = bt.first + bt.cands.size();
    {
      std::lock_guard<std::mutex> lk(mu);
      for (uint32_t w = 0; w < K; ++w) tables[w].thresholds(d.geoms[w].chi2_thr, &thr_wu[w * kNumHarmonicLevels]);
    }
    if (!bt.tin.empty()) {
      const TemplateInput& last = bt.tin.back();
      d.info.orbital_radius = last.tau;
      d.info.orbital_period = last.P;
      d.info.orbital_phase = last.Psi0;
    }
    uint32_t prefix = 0;
    while (next_block < blocks.size() && applied >= blocks[next_block].first) prefix = blocks[next_block++].second;
    if (hook && !hook(applied, prefix)) {
      res.interrupted = true;
      break;
    }
  }
  stop.store(true);
  for (auto& th : threads) th.join();
  res.t_templates += now_s() - t0;
  res.stats = stats();
  return rc;
}

int MultiSession::finalize(const std::vector<std::string>& outputs, uint32_t n_done,
                           std::vector<CandidateTable>& tables) {
  Impl& d = *impl_;
  if (outputs.size() != d.wus.size() || tables.size() != d.wus.size()) return RADPUL_EVAL;
  for (size_t k = 0; k < d.wus.size(); ++k) {
    SearchOptions o = d.opt;
    o.inputfile = d.inputs[k];
    o.outputfile = outputs[k];
    if (!o.checkpointfile.empty()) o.checkpointfile = d.opt.checkpointfile + "." + std::to_string(k);
    const int rc = finalize_output(o, d.geoms[k], n_done, tables[k], "einsteinbinary_mi355x");
    if (rc) return rc;
  }
  return 0;
}

}  // namespace brp
