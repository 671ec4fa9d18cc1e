"""NumPy model of the two-pass real-column plan (index math only).

N = N1 * N2 real samples x[n1 N2 + n2] (x = 0 for n1 >= N1/3):
  pass A: per column n2, the packed complex FFT of length N1/2 over
          z[m] = x[2m N2 + n2] + i x[(2m+1) N2 + n2], untangled to the real
          column spectrum C[k1], k1 = 0 .. N1/2 (rows)
  pass B: per row k1, Y[k2] = sum_n2 W_N^{k1 n2} C[k1][n2] W_N2^{n2 k2}
          = X[k1 + N1 k2]; power row P'[k1][k2]
  gather: P[k] = P'[r][k // N1]            if r = k mod N1 <= N1/2
               = P'[N1 - r][N2 - 1 - k // N1] otherwise (X[N-k] = conj X[k])
"""
import numpy as np


def model(x, N1, N2):
    N = N1 * N2
    H = N1 // 2
    cols = x.reshape(N1, N2)  # [n1][n2]
    z = cols[0::2, :] + 1j * cols[1::2, :]  # [m][n2], m < H
    Z = np.fft.fft(z, axis=0)  # [k][n2]
    k1 = np.arange(H + 1)[:, None]
    zk = Z[(k1 % H)[:, 0], :]
    zm = np.conj(Z[((H - k1) % H)[:, 0], :])
    w = np.exp(-2j * np.pi * k1 / N1)
    C = 0.5 * (zk + zm) - 0.5j * w * (zk - zm)  # [k1][n2], k1 = 0..H
    n2 = np.arange(N2)[None, :]
    A = C * np.exp(-2j * np.pi * k1 * n2 / N)
    Y = np.fft.fft(A, axis=1)  # [k1][k2]
    Pp = np.abs(Y) ** 2
    k = np.arange(N // 2 + 1)
    r = k % N1
    j = k // N1
    P = np.where(r <= H, Pp[np.minimum(r, H), np.minimum(j, N2 - 1)],
                 Pp[np.clip(N1 - r, 0, H), np.clip(N2 - 1 - j, 0, N2 - 1)])
    return P


if __name__ == "__main__":
    rng = np.random.default_rng(1)
    for N1, N2 in [(12, 8), (24, 16), (768, 64)]:
        N = N1 * N2
        x = np.zeros(N)
        x[: N // 3] = rng.standard_normal(N // 3)
        ref = np.abs(np.fft.rfft(x)) ** 2
        got = model(x, N1, N2)
        err = np.max(np.abs(got - ref)) / np.max(ref)
        print(f"N1={N1} N2={N2}: max rel err {err:.2e}")
        assert err < 1e-10
