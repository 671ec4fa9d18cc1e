"""Summarise a rocprofv3 --marker-trace CSV: count / total / mean ms per roctx range name.

usage: python3 scripts/marker_stats.py <marker_api_trace.csv>
"""
import csv
import sys
from collections import defaultdict


def main(path):
    rows = list(csv.DictReader(open(path)))
    if not rows:
        print("no marker rows")
        return
    cols = rows[0].keys()
    name_col = next((c for c in ("Message", "Marker_Name", "Name", "Function") if c in cols), None)
    start = next((c for c in cols if c.lower().startswith("start")), None)
    end = next((c for c in cols if c.lower().startswith("end")), None)
    if not (name_col and start and end):
        print("unknown columns:", list(cols))
        return
    agg = defaultdict(lambda: [0, 0.0])
    for r in rows:
        ms = (int(r[end]) - int(r[start])) * 1e-6
        a = agg[r[name_col]]
        a[0] += 1
        a[1] += ms
    print(f"{'range':32s} {'count':>7s} {'total ms':>11s} {'mean us':>10s}")
    for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{k:32s} {n:7d} {t:11.2f} {1e3 * t / n:10.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
