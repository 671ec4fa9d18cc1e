#include "cpu_fft.hpp"

#include <cmath>
#include <stdexcept>

namespace brp {

namespace {
std::vector<size_t> factorize(size_t n) {
  std::vector<size_t> f;
  while (n % 4 == 0) { f.push_back(4); n /= 4; }
  while (n % 2 == 0) { f.push_back(2); n /= 2; }
  for (size_t p = 3; p * p <= n; p += 2)
    while (n % p == 0) { f.push_back(p); n /= p; }
  if (n > 1) f.push_back(n);
  return f;
}

// exp(-2 pi i j / n) with the angle reduced exactly in integers
cd twiddle(size_t j, size_t n) {
  j %= n;
  // use symmetry to keep the argument small: angle = 2 pi j / n
  const long double a = -2.0L * 3.14159265358979323846264338327950288L * static_cast<long double>(j) /
                        static_cast<long double>(n);
  return cd(static_cast<double>(std::cos(a)), static_cast<double>(std::sin(a)));
}
}  // namespace

CpuFFT::CpuFFT(size_t n) : n_(n) {
  if (n == 0) throw std::invalid_argument("FFT size 0");
  factors_ = factorize(n);
  if (factors_.back() > kMaxDirectPrime) {
    // chirp w_j = exp(-pi i j^2 / n) with j^2 reduced mod 2n exactly
    size_t L = 1;
    while (L < 2 * n - 1) L <<= 1;
    chirp_.resize(n);
    for (size_t j = 0; j < n; ++j) {
      const unsigned __int128 jj = static_cast<unsigned __int128>(j) * j;
      chirp_[j] = twiddle(static_cast<size_t>(jj % (2 * n)), 2 * n);
    }
    conv_ = std::make_unique<CpuFFT>(L);
    hspec_.assign(L, cd(0, 0));
    hspec_[0] = std::conj(chirp_[0]);
    for (size_t j = 1; j < n; ++j) hspec_[j] = hspec_[L - j] = std::conj(chirp_[j]);
    conv_->forward(hspec_.data());
    return;
  }
  tw_.resize(n);
  for (size_t j = 0; j < n; ++j) tw_[j] = twiddle(j, n);
  scratch_.resize(n);
}

CpuFFT::~CpuFFT() = default;

// X_k = w_k sum_j (x_j w_j) conj(w_{k-j}): one forward and one inverse FFT of
// length L plus the precomputed spectrum of the conjugate chirp
void CpuFFT::bluestein(cd* data) {
  const size_t L = conv_->size();
  std::vector<cd> y(L, cd(0, 0));
  for (size_t j = 0; j < n_; ++j) y[j] = data[j] * chirp_[j];
  conv_->forward(y.data());
  for (size_t k = 0; k < L; ++k) y[k] *= hspec_[k];
  conv_->inverse(y.data());
  const double inv_l = 1.0 / static_cast<double>(L);
  for (size_t k = 0; k < n_; ++k) data[k] = y[k] * chirp_[k] * inv_l;
}

void CpuFFT::rec(const cd* in, size_t istride, cd* out, size_t n, size_t fac_idx, size_t tw_stride, bool inv) {
  if (n == 1) {
    out[0] = in[0];
    return;
  }
  const size_t p = factors_[fac_idx];
  const size_t m = n / p;
  for (size_t r = 0; r < p; ++r) rec(in + r * istride, istride * p, out + r * m, m, fac_idx + 1, tw_stride * p, inv);
  cd t[64];
  std::vector<cd> tbig;
  cd* tp = t;
  if (p > 64) {
    tbig.resize(p);
    tp = tbig.data();
  }
  for (size_t k = 0; k < m; ++k) {
    for (size_t r = 0; r < p; ++r) {
      cd w = tw_[(r * k * tw_stride) % n_];
      if (inv) w = std::conj(w);
      tp[r] = out[r * m + k] * w;
    }
    if (p == 2) {
      out[k] = tp[0] + tp[1];
      out[k + m] = tp[0] - tp[1];
    } else if (p == 4) {
      const cd a0 = tp[0] + tp[2], a1 = tp[0] - tp[2];
      const cd b0 = tp[1] + tp[3], b1 = tp[1] - tp[3];
      const cd jb1 = inv ? cd(-b1.imag(), b1.real()) : cd(b1.imag(), -b1.real());  // -i*b1 fwd
      out[k] = a0 + b0;
      out[k + m] = a1 + jb1;
      out[k + 2 * m] = a0 - b0;
      out[k + 3 * m] = a1 - jb1;
    } else {
      for (size_t q = 0; q < p; ++q) {
        cd s(0, 0);
        for (size_t r = 0; r < p; ++r) {
          cd w = tw_[((r * q) % p) * (n_ / p)];
          if (inv) w = std::conj(w);
          s += tp[r] * w;
        }
        out[k + q * m] = s;
      }
    }
  }
}

void CpuFFT::forward(cd* data) {
  if (conv_) return bluestein(data);
  rec(data, 1, scratch_.data(), n_, 0, 1, false);
  std::copy(scratch_.begin(), scratch_.end(), data);
}

void CpuFFT::inverse(cd* data) {
  if (conv_) {  // conj(DFT(conj x))
    for (size_t j = 0; j < n_; ++j) data[j] = std::conj(data[j]);
    bluestein(data);
    for (size_t j = 0; j < n_; ++j) data[j] = std::conj(data[j]);
    return;
  }
  rec(data, 1, scratch_.data(), n_, 0, 1, true);
  std::copy(scratch_.begin(), scratch_.end(), data);
}

void rfft_forward(const std::vector<double>& x, std::vector<cd>& X) {
  const size_t n = x.size();
  const size_t half = n / 2 + 1;
  X.assign(half, cd(0, 0));
  if (n % 2) {
    std::vector<cd> z(n);
    for (size_t i = 0; i < n; ++i) z[i] = cd(x[i], 0);
    CpuFFT(n).forward(z.data());
    for (size_t k = 0; k < half; ++k) X[k] = z[k];
    return;
  }
  const size_t m = n / 2;
  std::vector<cd> z(m);
  for (size_t i = 0; i < m; ++i) z[i] = cd(x[2 * i], x[2 * i + 1]);
  CpuFFT(m).forward(z.data());
  for (size_t k = 0; k <= m; ++k) {
    const cd zk = z[k % m];
    const cd zmk = std::conj(z[(m - k) % m]);
    const cd w = twiddle(k, n);
    const cd e = 0.5 * (zk + zmk);
    const cd o = cd(0, -0.5) * (zk - zmk);
    X[k] = e + w * o;
  }
}

void rfft_inverse(const std::vector<cd>& Xin, size_t n, std::vector<double>& x) {
  x.assign(n, 0.0);
  std::vector<cd> X(Xin);
  X[0] = cd(X[0].real(), 0);
  if (n % 2 == 0) X[n / 2] = cd(X[n / 2].real(), 0);
  if (n % 2) {
    std::vector<cd> z(n);
    // c2r of odd length reads bins 0 .. (n-1)/2 only (FFTW semantics)
    for (size_t k = 0; k < n; ++k) z[k] = (k <= n / 2) ? X[k] : std::conj(X[n - k]);
    CpuFFT(n).inverse(z.data());
    for (size_t i = 0; i < n; ++i) x[i] = z[i].real();
    return;
  }
  const size_t m = n / 2;
  std::vector<cd> z(m);
  for (size_t k = 0; k < m; ++k) {
    const cd a = X[k];
    const cd b = std::conj(X[m - k]);
    const cd winv = std::conj(twiddle(k, n));
    z[k] = (a + b) + cd(0, 1) * winv * (a - b);
  }
  CpuFFT(m).inverse(z.data());
  for (size_t i = 0; i < m; ++i) {
    x[2 * i] = z[i].real();
    x[2 * i + 1] = z[i].imag();
  }
}

}  // namespace brp
