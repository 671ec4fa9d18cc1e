// CPU golden backend wrapped in the Backend interface (plumbing path of
// BASELINE config 1; also the reference numerics for the HIP backend tests).
#include <algorithm>
#include <cmath>
#include <cstring>

#include "../core/cpu_backend.hpp"
#include "../core/resamp_math.hpp"
#include "backend.hpp"

namespace brp {

namespace {
class CpuEngine final : public Backend {
 public:
  const char* name() const override { return "cpu"; }
  int setup(const SearchGeometry& g, const SearchOptions& opt, std::vector<float>& series,
            const std::vector<ZapRange>& zaps) override {
    g_ = g;
    if (opt.white) {
      int rc = cpu_whiten(series, g, opt, zaps);
      if (rc) return rc;
    }
    series_ = series;
    return 0;
  }
  int process(const TemplateInput* t, int n, const float thr[kNumHarmonicLevels],
              std::vector<TemplateCands>& out) override {
    out.resize(n);
    std::vector<float> x, ps;
    for (int k = 0; k < n; ++k) {
      const ResampParams p = make_resamp_params(g_.nsamples, g_.n_unpadded, g_.fft_size, g_.dt, g_.step_inv,
                                                t[k].P, t[k].tau, t[k].Psi0);
      cpu_resample(series_.data(), p, x, nullptr, nullptr);
      cpu_power_spectrum(x, g_.fft_size, ps);
      cpu_harmonic_sum(ps, g_, thr, out[k].level);
    }
    stats_.templates += n;
    stats_.batches += 1;
    return 0;
  }
  int debug_buffers(const TemplateInput& t, std::vector<float>& series, std::vector<float>& ps) override {
    series = series_;
    const ResampParams p = make_resamp_params(g_.nsamples, g_.n_unpadded, g_.fft_size, g_.dt, g_.step_inv, t.P, t.tau,
                                              t.Psi0);
    std::vector<float> x;
    cpu_resample(series_.data(), p, x, nullptr, nullptr);
    cpu_power_spectrum(x, g_.fft_size, ps);
    return 0;
  }
  int preferred_batch() const override { return 1; }
  // queued submit/complete (Backend defaults), two deep: the search workers'
  // pipelined loop runs on the CPU golden model too
  int max_in_flight() const override { return 2; }
  BackendStats stats() const override { return stats_; }

 private:
  SearchGeometry g_;
  std::vector<float> series_;
  BackendStats stats_;
};

// Replay backend: no compute, returns `per_level` synthetic candidates per
// level and template (bins and powers derived from the template parameters,
// powers a little above the device threshold, so the in-order applier sees the
// insert/reject mix of a real search while the table fills). Used to measure
// what the applier thread sustains with many devices (BRP_REPLAY_BACKEND).
class ReplayEngine final : public Backend {
 public:
  ReplayEngine(int per_level, int batch) : per_level_(per_level), batch_(batch) {}
  const char* name() const override { return "replay"; }
  int setup(const SearchGeometry& g, const SearchOptions&, std::vector<float>&, const std::vector<ZapRange>&) override {
    g_ = g;
    return 0;
  }
  int process(const TemplateInput* t, int n, const float thr[kNumHarmonicLevels],
              std::vector<TemplateCands>& out) override {
    out.resize(n);
    for (int k = 0; k < n; ++k) {
      uint32_t bits;
      std::memcpy(&bits, &t[k].P, 4);
      uint64_t x = (static_cast<uint64_t>(bits) << 32) ^ static_cast<uint64_t>(t[k].Psi0 * 1e6f) ^ 0x9E3779B97F4A7C15ull;
      auto next = [&x] {
        x ^= x >> 12, x ^= x << 25, x ^= x >> 27;
        return x * 0x2545F4914F6CDD1Dull;
      };
      const uint32_t lo = g_.window_2, span = g_.fundamental_idx_hi > lo ? g_.fundamental_idx_hi - lo : 1;
      for (int h = 0; h < kNumHarmonicLevels; ++h) {
        std::vector<BinPower>& lv = out[k].level[h];
        lv.clear();
        for (int c = 0; c < per_level_; ++c) {
          const uint64_t r = next();
          const float u = static_cast<float>((r >> 40) & 0xFFFFFF) / 16777216.0f;
          lv.push_back(BinPower{lo + static_cast<uint32_t>(r % span), thr[h] * (1.0f + 0.5f * u * u * u)});
        }
      }
    }
    stats_.templates += n;
    stats_.batches += 1;
    return 0;
  }
  int preferred_batch() const override { return batch_; }
  int max_in_flight() const override { return 2; }  // as the HIP pipelines
  BackendStats stats() const override { return stats_; }

 private:
  int per_level_, batch_;
  SearchGeometry g_;
  BackendStats stats_;
};
}  // namespace

std::unique_ptr<Backend> make_cpu_backend() { return std::make_unique<CpuEngine>(); }
std::unique_ptr<Backend> make_replay_backend(int per_level, int batch) {
  return std::make_unique<ReplayEngine>(per_level, std::max(1, batch));
}

}  // namespace brp
