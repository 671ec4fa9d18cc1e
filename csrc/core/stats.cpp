#include "stats.hpp"

#include <cfloat>
#include <cmath>

namespace brp {

double log_chisq_Q_even(double x, int k) {
  if (x <= 0.0) return 0.0;
  const double y = 0.5 * x;
  // sum_{j<k} y^j/j!, accumulated with scaling to stay finite
  double term = 1.0, sum = 1.0;
  for (int j = 1; j < k; ++j) {
    term *= y / j;
    sum += term;
  }
  return -y + std::log(sum);
}

double chisq_Q_even(double x, int k) {
  if (x <= 0.0) return 1.0;
  const double y = 0.5 * x;
  double term = 1.0, sum = 1.0;
  for (int j = 1; j < k; ++j) {
    term *= y / j;
    sum += term;
  }
  const double e = std::exp(-y);
  if (e > 0.0 && std::isfinite(sum)) return e * sum;
  return std::exp(-y + std::log(sum));
}

double chisq_Qinv_even(double p, int k) {
  if (!(p > 0.0)) return INFINITY;
  if (p >= 1.0) return 0.0;
  const double logp = std::log(p);
  // bracket in y = x/2: Q is decreasing in y
  double lo = 0.0, hi = 1.0;
  while (log_chisq_Q_even(2.0 * hi, k) > logp) hi *= 2.0;
  double y = 0.5 * (lo + hi);
  for (int it = 0; it < 200; ++it) {
    const double lq = log_chisq_Q_even(2.0 * y, k);
    if (lq > logp) lo = y; else hi = y;
    // Newton step on g(y) = log Q(y) - log p, g'(y) = -pdf/Q
    // pdf/Q = y^(k-1)/(k-1)! / sum_{j<k} y^j/j!
    double term = 1.0, sum = 1.0;
    for (int j = 1; j < k; ++j) {
      term *= y / j;
      sum += term;
    }
    const double ratio = term / sum;  // term == y^(k-1)/(k-1)!
    double ynew = y + (lq - logp) / ratio;
    if (!(ynew > lo && ynew < hi)) ynew = 0.5 * (lo + hi);
    if (std::fabs(ynew - y) <= 1e-15 * y) {
      y = ynew;
      break;
    }
    y = ynew;
  }
  return 2.0 * y;
}

float single_bin_probability(float fA, unsigned fft_size) {
  return static_cast<float>(1.0 - std::pow(1.0 - static_cast<double>(fA), 1.0 / fft_size));
}

void power_thresholds(float prob, float thr[5]) {
  for (int h = 0; h < 5; ++h) {
    const int n_h = 1 << h;
    thr[h] = static_cast<float>(0.5 * chisq_Qinv_even(static_cast<double>(prob), n_h));
  }
}

double candidate_significance(double power, unsigned n_harm) {
  const double q = chisq_Q_even(2.0 * power, static_cast<int>(n_harm));
  if (q < DBL_MIN) return 320.0;
  return -std::log10(q);
}

}  // namespace brp
