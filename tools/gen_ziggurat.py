"""Regenerate csrc/core/ziggurat_tables.hpp.

GSL's gsl_ran_gaussian_ziggurat (used by the reference to fill zapped RFI bins,
demod_binary.c:1015-1021) samples a 128-layer ziggurat of f(x)=exp(-x^2/2).
GSL is not installed in this image, so the tables are rebuilt from the
construction: equal-area layers built from the top (y=1) downwards, the layer
area V chosen so that the 127th layer edge equals PARAM_R = 3.44428647676, and a
base strip of width V/f(R). The first entries reproduce GSL's published
12-digit values (ytab[1]=0.963598623011, ktab[1]=12590644,
wtab[0]=1.62318314817e-08, ...), see tests/test_rng.py.
"""
import math
import os

from scipy.optimize import brentq

R = 3.44428647676


def f(x):
    return math.exp(-0.5 * x * x)


def build(V):
    xs, ys, yt = [], [1.0], 1.0
    for _ in range(127):
        xi = brentq(lambda v: v * (yt - f(v)) - V, 1e-12, 20, xtol=1e-15, rtol=1e-15)
        xs.append(xi)
        yt = f(xi)
        ys.append(yt)
    return xs, ys


def main():
    V = brentq(lambda v: build(v)[0][126] - R, 9.9e-3, 9.92e-3, xtol=1e-18)
    xs, ys = build(V)
    xs.append(V / f(R))
    ytab = ys[:128]
    ktab = [0] + [int(2 ** 24 * xs[i - 1] / xs[i]) for i in range(1, 128)]
    wtab = [v * 2 ** -24 for v in xs]

    def rows(vals, fmt, per=4):
        return ",\n".join("    " + ", ".join(fmt(v) for v in vals[k:k + per])
                          for k in range(0, len(vals), per))

    out = os.path.join(os.path.dirname(__file__), "..", "csrc", "core", "ziggurat_tables.hpp")
    with open(out) as fh:
        head = fh.read().split("constexpr double kYTab")[0]
    body = (f"constexpr double kYTab[128] = {{\n{rows(ytab, lambda v: '%.12g' % v)}}};\n\n"
            f"constexpr unsigned long kKTab[128] = {{\n{rows(ktab, lambda v: '%dUL' % v)}}};\n\n"
            f"constexpr double kWTab[128] = {{\n{rows(wtab, lambda v: '%.12g' % v)}}};\n\n"
            "}  // namespace zig\n}  // namespace brp\n")
    with open(out, "w") as fh:
        fh.write(head + body)


if __name__ == "__main__":
    main()
