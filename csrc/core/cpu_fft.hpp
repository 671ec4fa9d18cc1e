// Double-precision mixed-radix FFT for the CPU golden backend.
//
// The reference's CPU backend uses FFTW (demod_binary_fft_fftw.c); this is a
// self-contained replacement for the host/golden path only. The product path
// on MI355X is the hand-written HIP FFT in csrc/hip/fft.hip.
#pragma once

#include <complex>
#include <cstddef>
#include <vector>

namespace brp {

using cd = std::complex<double>;

class CpuFFT {
 public:
  explicit CpuFFT(size_t n);
  size_t size() const { return n_; }
  // In-place complex DFT, forward = exp(-2 pi i nk/N), unnormalised.
  void forward(cd* data);
  void inverse(cd* data);

 private:
  void rec(const cd* in, size_t istride, cd* out, size_t n, size_t fac_idx, size_t tw_stride, bool inv);
  size_t n_;
  std::vector<size_t> factors_;
  std::vector<cd> tw_;  // exp(-2 pi i j / n)
  std::vector<cd> scratch_;
};

// Real -> half-complex (fft_size = N/2+1 outputs), unnormalised (FFTW r2c semantics).
void rfft_forward(const std::vector<double>& x, std::vector<cd>& X);
// Half-complex -> real (N outputs), unnormalised: returns N * x (FFTW c2r semantics);
// imaginary parts of X[0] and X[N/2] are ignored.
void rfft_inverse(const std::vector<cd>& X, size_t n, std::vector<double>& x);

}  // namespace brp
