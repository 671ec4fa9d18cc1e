#include "gsl_compat.hpp"

#include <cmath>

#include "ziggurat_tables.hpp"

namespace brp {

namespace {
inline uint32_t lcg(uint64_t n) { return static_cast<uint32_t>((69069ULL * n) & 0xffffffffULL); }

inline uint32_t taus_step(uint32_t s, int a, int b, uint32_t c, int d) {
  return ((s & c) << d) ^ (((s << a) ^ s) >> b);
}
}  // namespace

void Taus2::set(unsigned long seed) {
  uint64_t s = seed;
  if (s == 0) s = 1;  // GSL default seed
  s1_ = lcg(s);
  if (s1_ < 2) s1_ += 2;
  s2_ = lcg(s1_);
  if (s2_ < 8) s2_ += 8;
  s3_ = lcg(s2_);
  if (s3_ < 16) s3_ += 16;
  for (int i = 0; i < 6; ++i) get();  // warm-up, as GSL does
}

uint32_t Taus2::get() {
  s1_ = taus_step(s1_, 13, 19, 4294967294u, 12);
  s2_ = taus_step(s2_, 2, 25, 4294967288u, 4);
  s3_ = taus_step(s3_, 3, 11, 4294967280u, 17);
  return s1_ ^ s2_ ^ s3_;
}

double gaussian_ziggurat(Taus2& rng, double sigma) {
  unsigned long i, j;
  int sign;
  double x, y;
  for (;;) {
    // taus2 has a full 32-bit range: one draw gives the layer (low 8 bits,
    // bit 7 = sign) and a 24-bit abscissa.
    const unsigned long k = rng.get();
    i = k & 0xFF;
    j = (k >> 8) & 0xFFFFFF;
    sign = (i & 0x80) ? +1 : -1;
    i &= 0x7f;
    x = j * zig::kWTab[i];
    if (j < zig::kKTab[i]) break;
    if (i < 127) {
      const double y0 = zig::kYTab[i];
      const double y1 = zig::kYTab[i + 1];
      const double u1 = rng.uniform();
      y = y1 + (y0 - y1) * u1;
    } else {
      const double u1 = 1.0 - rng.uniform();
      const double u2 = rng.uniform();
      x = zig::kParamR - std::log(u1) / zig::kParamR;
      y = std::exp(-zig::kParamR * (x - zig::kParamR / 2)) * u2;
    }
    if (y < std::exp(-0.5 * x * x)) break;
  }
  return sign * sigma * x;
}

}  // namespace brp
