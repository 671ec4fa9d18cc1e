"""LDS bank-conflict model of two kernels' access patterns (gfx950 rules,
MI355X_MICROARCH.md §LDS): ds_read_b32 is serviced as 2 x 32 lanes on 32 banks,
ds_read_b64 as 2 x 32 lanes on 64 banks, ds_read2_b64 / ds_write2_b64 as
4 x 16 lanes on 32 banks; each extra distinct address on a bank within a group
costs one cycle. Prints extra cycles per wave for
  * the pruned harmonic sum's bound phase (csrc/hip/harmonic_sum.hip), round-2
    b32 cell reads vs the round-3 aligned pair reads, and
  * pass 3's last radix-16 stage twiddle reads (csrc/hip/fft_block.hpp) from the
    padded table vs the q-major block, and its untangle reads.
Usage: python tools/lds_bank_model.py"""

K_HARM = [16, 8, 12, 4, 14, 10, 6, 2, 15, 13, 11, 9, 7, 5, 3, 1]
CK = 3


def cell(L, K, i):
    return ((L * max(i, 0) + 8) >> 4) >> K


def extra_cycles(addrs, kind):
    if kind == "b32":
        groups, mod = [range(0, 32), range(32, 64)], 32
    elif kind == "b64":  # float2 units: 64 banks = 32 float2
        groups, mod = [range(0, 32), range(32, 64)], 32
    else:  # read2/write2_b64, float2 units on 32 dword banks
        groups, mod = [range(0, 16), range(16, 32), range(32, 48), range(48, 64)], 16
    ex = 0
    for g in groups:
        banks = {}
        for lane in g:
            a = addrs[lane]
            banks.setdefault(a % mod, set()).add(a)
        ex += max(len(v) for v in banks.values()) - 1
    return ex


def hs_bound(I0=488):
    old = new = 0
    for q, L in enumerate(K_HARM):
        K = CK if L >= 4 else 0
        tail = q < 8
        N = 20 if tail else 16
        span = (((L * (N - 1) + 15) // 16) >> K) + 2
        c0 = cell(L, K, I0)
        # round 2: b32 reads min(lo + d, hi) over the 16 indices, then the 4-index tail
        for n, off in ((16, 0), (4, 16)) if tail else ((16, 0),):
            kc = (((L * (n - 1) + 15) // 16) >> K) + 2
            for d in range(kc):
                addrs = []
                for lane in range(64):
                    ib = I0 + 16 * lane + off
                    lo, hi = cell(L, K, ib), cell(L, K, ib + n - 1)
                    addrs.append(min(lo + d, hi) - c0)
                old += extra_cycles(addrs, "b32")
        # round 3: aligned pairs (b64) except harmonic 3 (b32, stride 3 words)
        if L == 3:
            continue
        for j in range(span // 2 + 1):
            addrs = [((cell(L, K, I0 + 16 * lane) - (c0 & ~1)) >> 1) + j for lane in range(64)]
            new += extra_cycles(addrs, "b64")
    return old, new


def pass3(L=256, ROWS=8, TPC=16, PITCH=272):
    def idx(r, c):
        return c * PITCH + 4 * (c >> 1) + r + (r >> 4)

    tw0 = 2 * ROWS * PITCH + 4 * ROWS
    padded = qmajor = untangle = 0
    for wave in range(4):
        lanes = [wave * 64 + l for l in range(64)]
        for q in range(1, 16):
            a = [tw0 + (t % TPC) * q % L + (((t % TPC) * q % L) >> 4) for t in lanes]
            padded += extra_cycles(a, "b64")
            b = [tw0 + L + L // 16 + 1 + (q - 1) * 16 + t % TPC for t in lanes]
            qmajor += extra_cycles(b, "b64")
        for it in range(8):
            zk = [idx(t // ROWS + 32 * it, t % ROWS) for t in lanes]
            zm = [idx(L - 1 - (t // ROWS + 32 * it), ROWS + t % ROWS) for t in lanes]
            untangle += extra_cycles(zk, "b64") + extra_cycles(zm, "b64")
    return padded / 4, qmajor / 4, untangle / 4


if __name__ == "__main__":
    o, n = hs_bound()
    print(f"pruned harmonic sum bound phase, extra LDS cycles per wave: b32 cells {o}, aligned pairs {n}")
    p, q, u = pass3()
    print(f"pass 3 (L3 = 256), extra LDS cycles per wave: stage-2 twiddles padded {p:.0f}, q-major {q:.0f}; "
          f"untangle reads {u:.0f}")
