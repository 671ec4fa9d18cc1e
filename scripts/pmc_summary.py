"""Aggregate rocprofv3 --pmc counter CSVs per kernel (mean per dispatch)."""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmcs"
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", r.get("Kernel-Name", "?"))
        short = name.split("namespace)::")[-1].split("(")[0][:60]
        acc[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(acc):
    vals = {c: sum(v) / len(v) for c, v in acc[k].items()}
    print(k)
    for c in sorted(vals):
        print(f"    {c:28s} {vals[c]:16.1f}")
