// Host-side plan of the three-pass FFT used for every per-template transform.
//
// The real series of length N = 2M is transformed as an M-point complex FFT of
// z[n] = x[2n] + i x[2n+1] (packed real FFT), with M = L1*L2*L3:
//   input  index n = n1*(L2*L3) + n2*L3 + n3
//   output index k = k1 + L1*k2 + L1*L2*k3
// pass 1: L1-point FFTs over n1 (stride L2*L3), twiddle W_{L1 L2}^{n2 k1}
// pass 2: L2-point FFTs over n2 (stride L3),    twiddle W_M^{n3 (k1 + L1 k2)}
// pass 3: L3-point FFTs over n3 (contiguous rows), rows k1 + L1 k2 paired with
//         their mirror rows for the real-FFT untangle, natural-order output.
// Passes 1 and 2 are "column" passes over 16 adjacent columns (128-B rows).
#pragma once

#include <cstdint>

namespace brp {

struct FFTPlan3 {
  uint32_t M = 0;              // complex length (N/2)
  uint32_t L1 = 0, L2 = 0, L3 = 0;
  uint32_t ncol1 = 16, ncol2 = 16, rows3 = 8;  // columns / rows per workgroup
  uint32_t persist_wgs = 0;    // persistent passes: workgroups per launch (0: one per tile)
  uint32_t wg1() const { return (L2 * L3) / ncol1; }
  uint32_t wg2() const { return (L1 * L3) / ncol2; }
  // pass 3 (untangle): rows c in [0, C/2] with C = L1*L2
  uint32_t wg3() const { return ((L1 * L2) / 2 + rows3) / rows3; }
  // plain row pass (inverse transform): all C rows
  uint32_t wg3_plain() const { return (L1 * L2) / rows3; }
  bool valid() const { return M != 0 && L1 * L2 * L3 == M; }
};

// Chooses lengths from the instantiated kernel set; returns false if M is not
// supported (non-smooth length).
bool make_fft_plan(uint32_t M, FFTPlan3& plan);
// Plan of the convolution of a chirp-z transform of length Mb (any Mb): the
// smallest supported L >= 2 Mb - 1 (bluestein_kernels.hpp).
bool make_bluestein_plan(uint32_t Mb, FFTPlan3& plan);

}  // namespace brp
