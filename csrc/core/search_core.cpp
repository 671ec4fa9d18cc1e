#include "search_core.hpp"

#include <algorithm>
#include <cmath>
#include <cstring>

#include "errors.hpp"
#include "log.hpp"
#include "stats.hpp"

namespace brp {

int derive_geometry(const DDHeader& h, const SearchOptions& opt, SearchGeometry& g) {
  g.n_unpadded = h.nsamples;
  // (int)(uvar.padding*data_head.nsamples + 0.5): float product, double add
  const float padded = opt.padding * static_cast<float>(h.nsamples);
  g.nsamples = static_cast<uint32_t>(static_cast<int>(static_cast<double>(padded) + 0.5));
  g.t_obs_d = static_cast<double>(g.nsamples) * h.tsample * kMicrosec;
  g.t_obs = static_cast<float>(g.t_obs_d);
  g.dt = static_cast<float>(h.tsample * kMicrosec);
  g.step_inv = static_cast<float>(1.0 / g.dt);
  g.fft_size = static_cast<uint32_t>(g.nsamples * 0.5 + 0.5) + 1;
  g.window_2 = static_cast<uint32_t>(opt.window * 0.5 + 0.5);
  if (g.fft_size < opt.window) {
    log_message(LOG_ERROR, true, "Running median window (%u bins) is too wide for data set (%u bins)!\n",
                opt.window, g.fft_size);
    return RADPUL_EVAL;
  }
  const int lim = static_cast<int>(g.fft_size - g.window_2);
  const int f_hi = static_cast<int>(static_cast<double>(opt.f0 * g.t_obs) + 0.5);
  const int h_hi = static_cast<int>(16.0 * opt.f0 * g.t_obs + 0.5);
  g.fundamental_idx_hi = static_cast<uint32_t>(std::min(lim, f_hi));
  g.harmonic_idx_hi = static_cast<uint32_t>(std::min(lim, h_hi));
  g.nr_pages = (g.fundamental_idx_hi >> kLogPsPageSize) + 1;
  g.prob = single_bin_probability(opt.fA, g.fft_size);
  power_thresholds(g.prob, g.chi2_thr);
  return 0;
}

void CandidateTable::reset() { std::memset(c_, 0, sizeof(c_)); }

void CandidateTable::thresholds(const float chi2_thr[kNumHarmonicLevels], float thr[kNumHarmonicLevels]) const {
  for (int h = 0; h < kNumHarmonicLevels; ++h) {
    const float p = static_cast<float>(floor_power(h));
    thr[h] = std::fmax(p, chi2_thr[h]);
  }
}

void CandidateTable::insert_sorted(int h, int store_idx, uint32_t f0, float power, float P, float tau,
                                   float Psi0) {
  CPCand* lvl = c_ + h * kCandPerLevel;
  CPCand nc{};
  nc.f0 = f0;
  nc.P_b = P;
  nc.tau = tau;
  nc.Psi = Psi0;
  nc.power = power;
  nc.n_harm = 1u << h;
  nc.fA = lvl[store_idx].fA;
  // remove slot store_idx, then insert keeping the descending order; a new
  // entry goes after existing entries of equal power (stable sort semantics)
  const int s = store_idx - 0;
  std::memmove(lvl + s, lvl + s + 1, sizeof(CPCand) * (kCandPerLevel - 1 - s));
  int pos = 0;
  while (pos < kCandPerLevel - 1 && lvl[pos].power >= nc.power) ++pos;
  std::memmove(lvl + pos + 1, lvl + pos, sizeof(CPCand) * (kCandPerLevel - 1 - pos));
  lvl[pos] = nc;
}

int CandidateTable::apply_level(int h, const BinPower* bins, size_t n, float thr, float P, float tau, float Psi0) {
  CPCand* lvl = c_ + h * kCandPerLevel;
  int updates = 0;
  for (size_t k = 0; k < n; ++k) {
    const float power = bins[k].power;
    const uint32_t i = bins[k].bin;
    if (!(power > thr && power > lvl[kCandPerLevel - 1].power)) continue;
    int store_idx = kCandPerLevel - 1;
    for (int idx = 0; idx < kCandPerLevel; ++idx) {
      if (lvl[idx].f0 == i) {
        store_idx = (lvl[idx].power < power) ? idx : -1;
        break;
      }
    }
    if (store_idx >= 0) {
      insert_sorted(h, store_idx, i, power, P, tau, Psi0);
      ++updates;
    }
  }
  return updates;
}

void CandidateTable::merge(const CandidateTable& other) {
  for (int h = 0; h < kNumHarmonicLevels; ++h) {
    std::vector<CPCand> all;
    all.reserve(2 * kCandPerLevel);
    const CPCand* a = c_ + h * kCandPerLevel;
    const CPCand* b = other.c_ + h * kCandPerLevel;
    for (int k = 0; k < kCandPerLevel; ++k)
      if (a[k].n_harm) all.push_back(a[k]);
    for (int k = 0; k < kCandPerLevel; ++k) {
      if (!b[k].n_harm) continue;
      bool found = false;
      for (auto& e : all) {
        if (e.f0 == b[k].f0) {
          if (b[k].power > e.power) e = b[k];
          found = true;
          break;
        }
      }
      if (!found) all.push_back(b[k]);
    }
    std::stable_sort(all.begin(), all.end(), [](const CPCand& x, const CPCand& y) { return x.power > y.power; });
    CPCand* out = c_ + h * kCandPerLevel;
    std::memset(out, 0, sizeof(CPCand) * kCandPerLevel);
    for (size_t k = 0; k < all.size() && k < static_cast<size_t>(kCandPerLevel); ++k) out[k] = all[k];
  }
}

}  // namespace brp
