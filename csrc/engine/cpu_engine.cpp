// CPU golden backend wrapped in the Backend interface (plumbing path of
// BASELINE config 1; also the reference numerics for the HIP backend tests).
#include <cmath>

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
  int preferred_batch() const override { return 1; }
  BackendStats stats() const override { return stats_; }

 private:
  SearchGeometry g_;
  std::vector<float> series_;
  BackendStats stats_;
};
}  // namespace

std::unique_ptr<Backend> make_cpu_backend() { return std::make_unique<CpuEngine>(); }

}  // namespace brp
