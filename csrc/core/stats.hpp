// Chi-squared statistics for even degrees of freedom (2*N_h for N_h summed
// harmonics). The reference calls gsl_cdf_chisq_Q / gsl_cdf_chisq_Qinv
// (demod_binary.c:1161-1165, 1281, 1517-1548); for even dof both have a closed
// form, evaluated here in log space so no GSL is needed.
#pragma once

namespace brp {

// Upper tail Q(x; 2k) = exp(-x/2) * sum_{j<k} (x/2)^j / j!
double chisq_Q_even(double x, int k);
// log of the above (finite even where Q underflows)
double log_chisq_Q_even(double x, int k);
// Inverse: x such that Q(x; 2k) = p, for 0 < p < 1.
double chisq_Qinv_even(double p, int k);

// Single-bin false-alarm probability for an overall false alarm fA over
// fft_size bins, rounded to float as in the reference (demod_binary.c:1274).
float single_bin_probability(float fA, unsigned fft_size);

// Power thresholds thr[h] = 0.5*Qinv(prob, 2*2^h) as float (demod_binary.c:1281).
void power_thresholds(float prob, float thr[5]);

// -log10 of the false-alarm probability of a candidate with summed power P
// over n_harm harmonics; 320 when the probability underflows (below DBL_MIN, as
// GSL returns 0 there), demod_binary.c:1515-1551.
double candidate_significance(double power, unsigned n_harm);

}  // namespace brp
