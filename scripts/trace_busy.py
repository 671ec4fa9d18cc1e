"""GPU busy fraction and per-kernel time from a rocprofv3 kernel-trace CSV:
union of kernel intervals vs the traced span (timed region = last N dispatches)."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
# skip the warmup: keep the second half of the run (steps are identical)
iv = iv[len(iv) // 2:]
t0, t1 = iv[0][0], max(e for _, e, _ in iv)
busy, cur_s, cur_e = 0, None, None
for s, e, _ in iv:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
per = defaultdict(int)
for s, e, n in iv:
    per[n.replace("(anonymous namespace)::", "").split("(")[0][-60:]] += e - s
span = t1 - t0
print(f"span {span/1e6:.2f} ms  busy {busy/1e6:.2f} ms ({100*busy/span:.1f} %)  dispatches {len(iv)}")
for n, v in sorted(per.items(), key=lambda x: -x[1])[:10]:
    print(f"  {n:60s} {v/1e6:9.2f} ms (sum of durations)")
