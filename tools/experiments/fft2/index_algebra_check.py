import numpy as np
L1, R = 768, 8192
M = L1 * R
N = 2 * M
rng = np.random.default_rng(1)
nreal = 1 << 22
x = np.zeros(N); x[:nreal] = rng.standard_normal(nreal)
z = x[0::2] + 1j * x[1::2]
W = lambda n, e: np.exp(-2j * np.pi * (np.asarray(e) % n) / n)
# pass A: thread (c=n', j<16): x[q] = z[(j+16q) R + n'], q<16
Zc = z.reshape(L1, R)  # Zc[n1, n']
Y = np.zeros((L1, R), complex)
for s in range(3):
    st1 = np.zeros((256, R), complex)  # stage-1 outputs index 16 j + q'
    for j in range(16):
        xs = np.stack([Zc[j + 16 * q] * W(768, s * (j + 16 * q)) for q in range(16)])  # [q, n']
        y = np.fft.fft(xs, axis=0)  # DFT16 over q -> q'
        for qp in range(16):
            st1[16 * j + qp] = y[qp]
    for j in range(16):
        zz = np.stack([st1[j + 16 * q] * W(256, j * q) for q in range(16)])
        y = np.fft.fft(zz, axis=0)  # outputs k' = j + 16 q''
        for q2 in range(16):
            k1 = s + 3 * (j + 16 * q2)
            Y[k1] = y[q2] * W(M, np.arange(R) * k1)
# reference check of pass A: Y[k1][n'] = W_M^{n' k1} sum_n1 z[n1 R + n'] W_768^{n1 k1}
ref = np.fft.fft(Zc, axis=0) * W(M, np.outer(np.arange(L1), np.arange(R)))
print("pass A err", np.abs(Y - ref).max() / np.abs(ref).max())

def rowfft(row, jl_of_t):
    t = np.arange(512)
    # S1 radix 2: butterfly j1 < 4096: out[2 j1 + q]
    out = np.zeros(R, complex)
    a, b = row[:4096], row[4096:]
    out[0::2] = a + b; out[1::2] = a - b
    # S2 radix16 Ns2
    inp = out; out = np.zeros(R, complex)
    for tt in range(512):
        v = inp[tt + 512 * np.arange(16)] * (W(32, (tt % 2) * np.arange(16)))
        y = np.fft.fft(v)
        base = (tt // 2) * 32 + tt % 2
        out[base + 2 * np.arange(16)] = y
    # S3 radix16 Ns32 + writer-side S4 twiddle
    inp = out; out = np.zeros(R, complex)
    for tt in range(512):
        v = inp[tt + 512 * np.arange(16)] * W(512, (tt % 32) * np.arange(16))
        y = np.fft.fft(v)
        base = (tt // 32) * 512 + tt % 32
        e = base + 32 * np.arange(16)
        out[e] = y * W(8192, (e % 512) * (e // 512))
    # S4 radix 16 (no twiddle): thread tt -> butterfly jl
    res = np.zeros((512, 16), complex)
    for tt in range(512):
        jl = jl_of_t(tt)
        res[tt] = np.fft.fft(out[jl + 512 * np.arange(16)])  # X[jl + 512 q]
    return res

X = np.fft.fft(z)  # packed complex FFT
XM = np.abs(X).max()
Xr = np.fft.rfft(x)  # reference real FFT, bins 0..M
ps_ref = np.abs(Xr) ** 2 / N
ps = np.full(M + 1, np.nan)
for k1 in [0, 1, 5, 383, 384]:
    k1m = (L1 - k1) % L1
    row0 = k1 == 0
    self_ = row0 or k1 == 384
    va = rowfft(Y[k1], lambda tt: tt)
    vb = rowfft(Y[k1m], (lambda tt: (512 - tt) & 511) if row0 else (lambda tt: 511 - tt))
    # check va against direct
    for tt in range(512):
        for q in range(16):
            m = tt + 512 * q
            k = k1 + L1 * m
            zk = va[tt, q]
            pq = ((16 - q) & 15) if (row0 and tt == 0) else 15 - q
            zm = vb[tt, pq]
            assert abs(zk - X[k]) < 1e-6 * XM, (k1, tt, q)
            kk_expected = (M - k) % M
            assert abs(zm - X[kk_expected]) < 1e-6 * XM, ("mirror", k1, tt, q, kk_expected)
print("pass B row/mirror mapping OK")
