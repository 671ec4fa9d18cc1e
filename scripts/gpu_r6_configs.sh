#!/bin/bash
# Round 6: configs 5 (fp16 spectrum) and 4 (8 and 64 WUs resident) at HEAD, 1 GPU, bench.py JSON lines.
set -uo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/r6_cfg
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 200 python "$ROOT/bench.py" --steps 3 --warmup 1 --ps-fp16 > "$OUT/cfg5.json" 2> "$OUT/cfg5.err" || { echo "cfg5 failed"; tail -20 "$OUT/cfg5.err"; exit 1; }
timeout -k 10 300 python "$ROOT/bench.py" --steps 2 --warmup 1 --wus 8 > "$OUT/cfg4_8.json" 2> "$OUT/cfg4_8.err" || { echo "cfg4 8 failed"; tail -20 "$OUT/cfg4_8.err"; exit 1; }
timeout -k 10 600 python "$ROOT/bench.py" --steps 1 --warmup 1 --wus 64 > "$OUT/cfg4_64.json" 2> "$OUT/cfg4_64.err" || { echo "cfg4 64 failed"; tail -20 "$OUT/cfg4_64.err"; exit 1; }
for f in cfg5 cfg4_8 cfg4_64; do
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['recall_vs_golden'], d['dtype'], d['config']['work_units'])" "$OUT/$f.json" $f
done
