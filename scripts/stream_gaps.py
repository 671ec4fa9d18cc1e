"""Per-stream gaps between consecutive kernels of a rocprofv3 kernel trace
(run_kernel_trace.csv): how long each queue sits idle between the end of one
kernel and the start of the next, split by the kernel that follows, and the
share of the traced span each queue is busy.  python3 scripts/stream_gaps.py <csv>"""
import collections
import re
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
by_q = collections.defaultdict(list)
for r in rows:
    by_q[(r["Queue_Id"], r["Stream_Id"])].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
t0 = min(int(r["Start_Timestamp"]) for r in rows)
t1 = max(int(r["End_Timestamp"]) for r in rows)
print(f"span {(t1 - t0) / 1e6:.1f} ms, {len(rows)} kernels")
for q, ks in sorted(by_q.items()):
    ks.sort()
    if len(ks) < 100:
        continue
    busy = sum(e - s for s, e, _ in ks)
    gaps = collections.defaultdict(list)
    for (s0, e0, n0), (s1, e1, n1) in zip(ks, ks[1:]):
        g = s1 - e0
        if 0 <= g < 200_000:  # ignore long host-side stalls (> 200 us)
            gaps[re.sub(r"^.*::", "", n1.split("(anonymous namespace)::")[-1].split("(")[0])[:40]].append(g)
    span = ks[-1][1] - ks[0][0]
    print(f"queue {q}: {len(ks)} kernels, busy {busy / span * 100:.1f} % of its span")
    for n, g in sorted(gaps.items(), key=lambda kv: -sum(kv[1])):
        g.sort()
        pct = lambda f: g[min(len(g) - 1, int(f * len(g)))] / 1e3
        print(f"   before {n:42s} n={len(g):6d} p10 {pct(.1):6.2f} median {pct(.5):6.2f} p90 {pct(.9):6.2f} us"
              f"  mean {sum(g) / len(g) / 1e3:6.2f} us  total {sum(g) / 1e6:6.1f} ms")
