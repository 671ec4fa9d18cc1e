// Double-precision mixed-radix FFT for the CPU golden backend.
//
// The reference's CPU backend uses FFTW (demod_binary_fft_fftw.c); this is a
// self-contained replacement for the host/golden path only. The product path
// on MI355X is the hand-written HIP FFT in csrc/hip/fft.hip.
#pragma once

#include <complex>
#include <cstddef>
#include <memory>
#include <vector>

namespace brp {

using cd = std::complex<double>;

class CpuFFT {
 public:
  explicit CpuFFT(size_t n);
  ~CpuFFT();
  size_t size() const { return n_; }
  // In-place complex DFT, forward = exp(-2 pi i nk/N), unnormalised.
  void forward(cd* data);
  void inverse(cd* data);

 private:
  void rec(const cd* in, size_t istride, cd* out, size_t n, size_t fac_idx, size_t tw_stride, bool inv);
  void bluestein(cd* data);
  size_t n_;
  std::vector<size_t> factors_;
  std::vector<cd> tw_;  // exp(-2 pi i j / n)
  std::vector<cd> scratch_;
  // Lengths with a prime factor above kMaxDirectPrime (any padding -P of the
  // reference gives such N) run as a chirp-z convolution (Bluestein) over a
  // power-of-two FFT of length >= 2n - 1, in double precision.
  static constexpr size_t kMaxDirectPrime = 64;
  std::unique_ptr<CpuFFT> conv_;  // length-L transform of the convolution
  std::vector<cd> chirp_;    // exp(-pi i j^2 / n), j < n
  std::vector<cd> hspec_;    // FFT_L of the conjugate chirp, wrapped
};

// Real -> half-complex (fft_size = N/2+1 outputs), unnormalised (FFTW r2c semantics).
void rfft_forward(const std::vector<double>& x, std::vector<cd>& X);
// Half-complex -> real (N outputs), unnormalised: returns N * x (FFTW c2r semantics);
// imaginary parts of X[0] and X[N/2] are ignored.
void rfft_inverse(const std::vector<cd>& X, size_t n, std::vector<double>& x);

}  // namespace brp
