"""Start-up timeline of a traced process from rocprofv3 --hip-trace --kernel-trace
CSVs: every HIP API call longer than a threshold (offset from the first traced
event, duration, thread), per-function totals, and the first / last kernel.
usage: python scripts/api_timeline.py <dir with *_hip_api_trace.csv> [min_ms]"""
import csv
import glob
import sys
from collections import defaultdict


def rows(pattern):
    out = []
    for p in glob.glob(pattern, recursive=True):
        with open(p) as f:
            out += list(csv.DictReader(f))
    return out


def main():
    d = sys.argv[1]
    min_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    api = rows(f"{d}/**/*hip_api_trace.csv")
    ker = rows(f"{d}/**/*kernel_trace.csv")
    if not api:
        print("no hip_api_trace.csv under", d)
        return
    t0 = min(int(r["Start_Timestamp"]) for r in api + ker)
    tot = defaultdict(lambda: [0, 0.0])
    long_calls = []
    for r in api:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        ms = (e - s) / 1e6
        t = tot[r["Function"]]
        t[0] += 1
        t[1] += ms
        if ms >= min_ms:
            long_calls.append(((s - t0) / 1e6, ms, r["Function"], r.get("Thread_Id", "")))
    print(f"HIP API calls >= {min_ms} ms (offset from the first traced event):")
    for off, ms, fn, tid in sorted(long_calls):
        print(f"  t={off:9.2f} ms  {ms:8.2f} ms  {fn}  thread {tid}")
    print("per-function totals (top 20 by time):")
    for fn, (n, ms) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:20]:
        print(f"  {fn:40s} calls={n:7d}  total={ms:9.2f} ms")
    if ker:
        ks = sorted(int(r["Start_Timestamp"]) for r in ker)
        ke = max(int(r["End_Timestamp"]) for r in ker)
        print(f"kernels: {len(ker)}; first starts at t={(ks[0] - t0) / 1e6:.2f} ms, last ends at t={(ke - t0) / 1e6:.2f} ms")
    last_api = max(int(r["End_Timestamp"]) for r in api)
    print(f"last API call ends at t={(last_api - t0) / 1e6:.2f} ms")


if __name__ == "__main__":
    main()
