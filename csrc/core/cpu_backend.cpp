#include "cpu_backend.hpp"

#include <cmath>
#include <cstdlib>
#include <cstring>

#include "cpu_fft.hpp"
#include "errors.hpp"
#include "gsl_compat.hpp"
#include "log.hpp"
#include "rngmed.hpp"

namespace brp {

void cpu_resample(const float* series, const ResampParams& p, std::vector<float>& out, uint32_t* n_steps_out,
                  float* mean_out) {
#pragma clang fp contract(off)
  const uint32_t nu = p.nsamples_unpadded;
  std::vector<float> del_t(nu);
  for (uint32_t i = 0; i < nu; ++i) del_t[i] = resamp_del_t(i, p, kSinLut, kCosLut);
  uint32_t n_steps = nu - 1;
  while (resamp_beyond_end(n_steps, del_t[n_steps], nu)) n_steps--;
  out.assign(p.nsamples, 0.0f);
  float mean = 0.0f;
  double dsum = 0.0;
  uint32_t i = 0;
  for (; i < n_steps; ++i) {
    int idx = resamp_nearest(i, del_t[i]);
    if (idx < 0) idx = 0;  // cannot happen for sane banks; keep the gather in bounds
    out[i] = series[idx];
    mean += out[i];
    dsum += out[i];
  }
  mean /= static_cast<float>(n_steps);
  // The reference's CPU build pads with this serial float mean
  // (demod_binary_resamp_cpu.c:113-125); its CUDA build reduces in a float
  // tree (cuda/app/demod_binary_cuda.cuh:123-150), and the MI355X pipeline in
  // double: on a raw (unwhitened) series of ~5e4 per sample the serial float
  // sum is off by up to ~2 %, which moves the low bins of the spectrum. The
  // golden model keeps the CPU build's value unless BRP_CPU_MEAN=double asks
  // for the accurate one (GPU / CUDA semantics, raw-series comparisons).
  const bool accurate = std::getenv("BRP_CPU_MEAN") && std::strcmp(std::getenv("BRP_CPU_MEAN"), "double") == 0;
  if (accurate) mean = static_cast<float>(dsum / static_cast<double>(n_steps));
  for (; i < p.nsamples; ++i) out[i] = mean;
  if (n_steps_out) *n_steps_out = n_steps;
  if (mean_out) *mean_out = mean;
}

void cpu_power_spectrum(const std::vector<float>& x, uint32_t fft_size, std::vector<float>& ps) {
  std::vector<double> xd(x.begin(), x.end());
  std::vector<cd> X;
  rfft_forward(xd, X);
  const double norm = static_cast<double>(1.0f / static_cast<float>(x.size()));
  ps.assign(fft_size, 0.0f);
  for (uint32_t k = 1; k < fft_size && k < X.size(); ++k) {
    const double re = static_cast<float>(X[k].real());
    const double im = static_cast<float>(X[k].imag());
    ps[k] = static_cast<float>(norm * (re * re + im * im));
  }
  ps[0] = 0.0f;
}

void cpu_harmonic_sum(const std::vector<float>& ps, const SearchGeometry& g, const float thr[kNumHarmonicLevels],
                      std::vector<BinPower> out[kNumHarmonicLevels], std::vector<float>* sumspec) {
#pragma clang fp contract(off)
  const uint32_t w2 = g.window_2, fhi = g.fundamental_idx_hi, hhi = g.harmonic_idx_hi;
  std::vector<float> ss[kNumHarmonicLevels];
  for (int h = 1; h < kNumHarmonicLevels; ++h) ss[h].assign(fhi, 0.0f);
  std::vector<uint8_t> hit[kNumHarmonicLevels];
  for (int h = 0; h < kNumHarmonicLevels; ++h) hit[h].assign(fhi, 0);
  const float* P = ps.data();
  uint32_t idx16[16];
  for (uint32_t l = 0; l < 16; ++l) idx16[l] = w2 * l + 8;
  int jprev[kNumHarmonicLevels] = {-1, -1, -1, -1, -1};
  float runmax[kNumHarmonicLevels] = {0, 0, 0, 0, 0};
  for (uint32_t i = w2; i < hhi; ++i) {
    float sum = P[i];
    if (sum > thr[0] && i < fhi) hit[0][i] = 1;
    auto level = [&](int h, int j) {
      if (j != jprev[h]) runmax[h] = 0.0f;
      if (static_cast<uint32_t>(j) < fhi) {
        const float power = (sum > runmax[h]) ? sum : runmax[h];
        if (power > thr[h]) {
          ss[h][j] = power;
          hit[h][j] = 1;
        } else if (j != jprev[h]) {
          ss[h][j] = power;
        }
        runmax[h] = power;
      }
      jprev[h] = j;
    };
    int j = static_cast<int>(idx16[8] >> 4);
    sum += P[j];
    level(1, j);
    j = static_cast<int>(idx16[4] >> 4);
    sum += P[idx16[12] >> 4] + P[j];
    level(2, j);
    j = static_cast<int>(idx16[2] >> 4);
    sum += P[idx16[14] >> 4] + P[idx16[10] >> 4] + P[idx16[6] >> 4] + P[j];
    level(3, j);
    j = static_cast<int>(idx16[1] >> 4);
    sum += P[idx16[15] >> 4] + P[idx16[13] >> 4] + P[idx16[11] >> 4] + P[idx16[9] >> 4] + P[idx16[7] >> 4] +
           P[idx16[5] >> 4] + P[idx16[3] >> 4] + P[j];
    level(4, j);
    for (uint32_t l = 0; l < 16; ++l) idx16[l] += l;
  }
  for (int h = 0; h < kNumHarmonicLevels; ++h) {
    out[h].clear();
    for (uint32_t b = w2; b < fhi; ++b) {
      if (!hit[h][b]) continue;
      const float v = (h == 0) ? P[b] : ss[h][b];
      if (v > thr[h]) out[h].push_back({b, v});
    }
  }
  if (sumspec) {
    sumspec->assign(static_cast<size_t>(kNumHarmonicLevels) * fhi, 0.0f);
    for (uint32_t b = 0; b < fhi; ++b) (*sumspec)[b] = P[b];
    for (int h = 1; h < kNumHarmonicLevels; ++h)
      std::memcpy(sumspec->data() + static_cast<size_t>(h) * fhi, ss[h].data(), fhi * sizeof(float));
  }
}

void make_zap_noise(int32_t seed, const SearchGeometry& g, const SearchOptions& opt,
                    const std::vector<ZapRange>& zaps, ZapNoise& noise) {
  noise.bin.clear();
  noise.re.clear();
  noise.im.clear();
  Taus2 rng(static_cast<unsigned long>(static_cast<long>(seed)));
  const double sigma = M_SQRT1_2 * static_cast<double>(std::sqrt(opt.padding));
  for (const auto& z : zaps) {
    const uint32_t lo = static_cast<uint32_t>(z.fmin * g.t_obs_d + 0.5);
    const uint32_t hi = static_cast<uint32_t>(z.fmax * g.t_obs_d + 0.5);
    for (uint32_t idx = lo; idx <= hi; ++idx) {
      const float re = static_cast<float>(gaussian_ziggurat(rng, sigma));
      const float im = static_cast<float>(gaussian_ziggurat(rng, sigma));
      noise.bin.push_back(idx);
      noise.re.push_back(re);
      noise.im.push_back(im);
      if (idx == 0xffffffffu) break;
    }
  }
}

int cpu_whiten(std::vector<float>& series, const SearchGeometry& g, const SearchOptions& opt,
               const std::vector<ZapRange>& zaps) {
  const uint32_t n = g.nsamples, fft_size = g.fft_size, window = opt.window;
  if (fft_size < window) return RADPUL_EVAL;
  int32_t seed;
  std::memcpy(&seed, series.data(), sizeof(seed));
  log_message(LOG_INFO, true, "Seed for random number generator is %d.\n", seed);
  std::vector<double> x(n, 0.0);
  for (uint32_t i = 0; i < g.n_unpadded; ++i) x[i] = series[i];
  std::vector<cd> X;
  rfft_forward(x, X);
  // odd N: fft_size = (N+1)/2 + 1 reaches one bin past the r2c output (the
  // reference reads an unwritten FFTW slot there); use the DFT's own value,
  // X_{(N+1)/2} = conj(X_{(N-1)/2})
  while (X.size() < fft_size) X.push_back(std::conj(X[n - X.size()]));
  // fft in single precision like the reference buffers
  std::vector<float> re(fft_size), im(fft_size);
  for (uint32_t k = 0; k < fft_size; ++k) {
    re[k] = static_cast<float>(X[k].real());
    im[k] = static_cast<float>(X[k].imag());
  }
  std::vector<float> ps(fft_size, 0.0f);
  for (uint32_t k = 1; k < fft_size; ++k) {
    const double a = re[k], b = im[k];
    ps[k] = static_cast<float>(a * a + b * b);
  }
  const uint32_t white_size = fft_size - window + 1;
  std::vector<float> med(white_size);
  running_median(ps.data(), fft_size, window, med.data());
  const uint32_t w2 = static_cast<uint32_t>(window * 0.5 + 0.5);
  for (uint32_t i = 0; i < white_size; ++i) {
    const float factor = static_cast<float>(std::sqrt(M_LN2 / med[i]));
    re[i + w2] *= factor;
    im[i + w2] *= factor;
  }
  ZapNoise noise;
  make_zap_noise(seed, g, opt, zaps, noise);
  for (size_t k = 0; k < noise.bin.size(); ++k) {
    if (noise.bin[k] < fft_size) {
      re[noise.bin[k]] = noise.re[k];
      im[noise.bin[k]] = noise.im[k];
    }
  }
  for (uint32_t i = 0; i < w2; ++i) {
    re[i] = im[i] = 0.0f;
    re[fft_size - i - 1] = im[fft_size - i - 1] = 0.0f;
  }
  for (uint32_t k = 0; k < fft_size; ++k) X[k] = cd(re[k], im[k]);
  std::vector<double> xt;
  rfft_inverse(X, n, xt);
  const float norm = static_cast<float>(1.0 / std::sqrt(static_cast<float>(n)));
  for (uint32_t i = 0; i < g.n_unpadded; ++i) series[i] = norm * static_cast<float>(xt[i]);
  return 0;
}

}  // namespace brp
