"""Per-step timeline of a bench run from a rocprofv3 kernel-trace CSV.

A step starts with the whitening kernels (whiten_power_kernel marks it) and
runs the template kernels until the next step's whitening. For every step:
whitening span (first whitening-phase kernel to the first template pass 1),
template span, GPU busy fraction (union of kernel intervals) over the whole
template span and over its first and last `edge` microseconds, and the idle
gap between the last template kernel and the next step. The ramp and tail
of a short (sharded) step are what its per-template rate loses against the
whole bank.

  python scripts/step_timeline.py <kernel_trace.csv> [edge_us=1000]
"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
edge = float(sys.argv[2]) * 1e3 if len(sys.argv) > 2 else 1e6
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
TEMPLATE = ("pass1_pruned3_kernel", "pass2r_kernel", "pass3_kernel", "hs_cells_kernel", "hs_pruned_kernel",
            "harmonic_sum_kernel", "pass2_kernel", "hs_sel_")


def is_template(name: str) -> bool:
    return any(k in name for k in TEMPLATE) and "pass1_kernel<" not in name


def busy(ivs, lo, hi):
    tot, cs, ce = 0, None, None
    for s, e in sorted((max(s, lo), min(e, hi)) for s, e, _ in ivs if e > lo and s < hi):
        if ce is None or s > ce:
            if ce is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if ce is not None:
        tot += ce - cs
    return tot


starts = [i for i, (_, _, n) in enumerate(iv) if "whiten_power_kernel" in n]
print(f"{len(starts)} steps")
print("step  whiten_us  templ_ms  busy%  first%  last%  tail_gap_us  kernels")
for k, i0 in enumerate(starts):
    i1 = starts[k + 1] if k + 1 < len(starts) else len(iv)
    seg = iv[i0:i1]
    # whitening begins at the first kernel after the previous step's template kernels
    j = i0
    while j > 0 and not is_template(iv[j - 1][2]) and (k == 0 or j - 1 >= starts[k - 1]):
        j -= 1
    w0 = iv[j][0]
    tmpl = [x for x in seg if is_template(x[2])]
    if not tmpl:
        continue
    t0 = tmpl[0][0]
    t1 = max(e for _, e, _ in tmpl)
    span = t1 - t0
    b = busy(tmpl, t0, t1)
    bf = busy(tmpl, t0, min(t1, t0 + edge))
    bl = busy(tmpl, max(t0, t1 - edge), t1)
    nxt = iv[i1][0] if i1 < len(iv) else t1
    w = min(edge, span)
    print(f"{k:4d}  {(t0 - w0) / 1e3:9.1f}  {span / 1e6:8.3f}  {100 * b / span:5.1f}  {100 * bf / w:6.1f}  "
          f"{100 * bl / w:5.1f}  {(nxt - t1) / 1e3:11.1f}  {len(tmpl)}")
