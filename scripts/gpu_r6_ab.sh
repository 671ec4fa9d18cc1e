#!/bin/bash
# Interleaved A/B of an engine switch on the headline bench (bench.py, 1 GPU):
#   scripts/gpu_r6_ab.sh VAR "VAL_A VAL_B" [rounds] [steps] [outdir]
# e.g. scripts/gpu_r6_ab.sh BRP_P3_CELLS "0 1" 3 5
# Each round runs every value once (A, B, A, B, ...), so box drift hits both;
# one JSON line per run in $OUT/ab_<VAR>.jsonl, a summary at the end.
set -uo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
VAR=$1
VALS=$2
ROUNDS=${3:-3}
STEPS=${4:-5}
OUT=${5:-$ROOT/gpurun_out/r6_ab}
mkdir -p "$OUT"
J=$OUT/ab_${VAR}.jsonl
: > "$J"
for r in $(seq 1 "$ROUNDS"); do
  for v in $VALS; do
    line=$(env "$VAR=$v" timeout -k 10 180 python "$ROOT/bench.py" --steps "$STEPS" --warmup 1 2> "$OUT/ab_${VAR}_${v}_$r.err" | grep '^{') || { echo "run $VAR=$v round $r failed"; tail -20 "$OUT/ab_${VAR}_${v}_$r.err"; exit 1; }
    echo "{\"var\": \"$VAR\", \"val\": \"$v\", \"round\": $r, \"bench\": $line}" >> "$J"
    echo "$VAR=$v round $r: $(echo "$line" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["recall_vs_golden"], d["table_identical_to_warmup"])')"
  done
done
python3 - "$J" <<'PY'
import json, sys, collections
rows = [json.loads(l) for l in open(sys.argv[1])]
by = collections.defaultdict(list)
sha = collections.defaultdict(set)
for r in rows:
    by[r["val"]].append(r["bench"]["value"])
    sha[r["val"]].add(r["bench"]["table_sha256"])
for v, xs in by.items():
    print(f"{rows[0]['var']}={v}: " + " / ".join(f"{x:.0f}" for x in xs) + f"  mean {sum(xs)/len(xs):.0f}  tables {sorted(sha[v])}")
PY
