// Bit-compatible replacements for the two GSL random-number facilities the
// reference uses for RFI zapping (demod_binary.c:989-1021):
//   gsl_rng_taus2              -> Taus2
//   gsl_ran_gaussian_ziggurat  -> gaussian_ziggurat()
// GSL is not available on MI355X build hosts, and the zapped bins must get the
// same noise for results to validate against other hosts.
#pragma once

#include <cstdint>

namespace brp {

// L'Ecuyer maximally-equidistributed combined Tausworthe generator with the
// "taus2" seeding procedure. Produces 32-bit outputs.
class Taus2 {
 public:
  explicit Taus2(unsigned long seed = 1) { set(seed); }
  void set(unsigned long seed);
  uint32_t get();
  // uniform in [0,1)
  double uniform() { return get() / 4294967296.0; }

 private:
  uint32_t s1_ = 0, s2_ = 0, s3_ = 0;
};

// Gaussian deviate with standard deviation sigma (Marsaglia-Tsang ziggurat with
// GSL's 128-layer tables and tail handling).
double gaussian_ziggurat(Taus2& rng, double sigma);

}  // namespace brp
