#!/bin/bash
# HIP start-up / exit cost under runtime environment settings (round 6):
# build/startup_bench (tools/experiments/startup/startup_bench.hip: runtime init,
# 3 streams with a buffer, first copy and kernel each, _exit) in fresh processes,
# the variants interleaved, R rounds; process wall time and exit time from the
# epoch stamp the program prints just before _exit.
# Usage: scripts/gpu_r6_startup_env.sh [rounds] [outfile] [VAR=value ...]
set -uo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
R=${1:-3}
OUT=${2:-$ROOT/gpurun_out/r6_startup_env.jsonl}
: > "$OUT"
shift 2 2>/dev/null || true
VARIANTS=("$@")
[ ${#VARIANTS[@]} -eq 0 ] && VARIANTS=("DEFAULT=1" "HSA_ENABLE_SDMA=0" "GPU_MAX_HW_QUEUES=2" "GPU_MAX_HW_QUEUES=1"
  "ROCR_VISIBLE_DEVICES=0" "HIP_FORCE_DEV_KERNARG=1" "AMD_DIRECT_DISPATCH=0" "HSA_ENABLE_INTERRUPT=0")
for r in $(seq 1 "$R"); do
  for v in "${VARIANTS[@]}"; do
    t0=$(date +%s%N)
    line=$(env "$v" timeout -k 5 60 "$ROOT/build/startup_bench" seq 3 none 80 2>/dev/null | grep '^{') || { echo "variant $v failed"; exit 1; }
    t1=$(date +%s%N)
    python3 - "$v" "$r" "$t0" "$t1" "$line" >> "$OUT" <<'PY'
import json, sys
v, r, t0, t1, line = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]) / 1e6, int(sys.argv[4]) / 1e6, sys.argv[5]
d = json.loads(line)
d.update(variant=v, round=r, process_ms=round(t1 - t0, 1), exit_ms=round(t1 - d["epoch_ms_before_exit"], 1))
print(json.dumps(d))
PY
  done
done
python3 - "$OUT" <<'PY'
import json, sys, collections
rows = [json.loads(l) for l in open(sys.argv[1])]
by = collections.defaultdict(list)
for d in rows: by[d["variant"]].append(d)
print(f"{'variant':26s} {'init':>18s} {'streams':>18s} {'exit':>18s} {'process':>20s}")
for v, ds in by.items():
    f = lambda k: " / ".join(f"{d[k]:.0f}" for d in ds)
    print(f"{v:26s} {f('init_ms'):>18s} {f('pipes_ms'):>18s} {f('exit_ms'):>18s} {f('process_ms'):>20s}")
PY
