#!/bin/bash
# The application on the reference protocol (scripts/bench_single.sh, BRP_PHASES=1)
# under HIP runtime environment settings, interleaved, R rounds (round 6): whole-
# process wall, template-loop time, exit after the last phase, result identity.
# Usage: scripts/gpu_r6_app_env.sh [rounds] [outdir] [variant ...]
set -uo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
R=${1:-3}
OUT=${2:-$ROOT/gpurun_out/r6_app_env}
shift 2 2>/dev/null || true
mkdir -p "$OUT" && OUT=$(cd "$OUT" && pwd)
VARIANTS=("$@")
[ ${#VARIANTS[@]} -eq 0 ] && VARIANTS=("NONE=1" "AMD_DIRECT_DISPATCH=0" "HSA_ENABLE_INTERRUPT=0" "AMD_DIRECT_DISPATCH=0 HSA_ENABLE_INTERRUPT=0")
export TMPDIR=/tmp
: > "$OUT/summary.txt"
for r in $(seq 1 "$R"); do
  k=0
  for v in "${VARIANTS[@]}"; do
    k=$((k + 1))
    W=/tmp/r6_env_${k}_$r
    rm -rf "$W"
    env $v BRP_PHASES=1 WORK=$W timeout -k 10 120 "$ROOT/scripts/bench_single.sh" > "$OUT/run_${k}_$r.txt" 2>&1 || { echo "variant '$v' round $r failed"; cat "$OUT/run_${k}_$r.txt"; exit 1; }
    grep -v '^% Date:' "$W/results.cand" > "$OUT/results_${k}_$r.cand"
    grep '\[phase\]' "$W/app.log" | sed 's/  epoch_ms=.*//' >> "$OUT/run_${k}_$r.txt"
    wall=$(grep -o 'in [0-9.]* s wall' "$OUT/run_${k}_$r.txt" | grep -o '[0-9.]*')
    loop=$(grep -o 'templates in [0-9.]* s (' "$W/app.log" | grep -o '[0-9.]*' | head -1)
    ex=$(grep -o "to exit [0-9.]* ms" "$OUT/run_${k}_$r.txt" | grep -o '[0-9.]*')
    up=$(grep 'HIP runtime up' "$W/app.log" | grep -o 't= *[0-9.]*' | grep -o '[0-9.]*')
    ps=$(grep 'pipelines set up' "$W/app.log" | grep -o 't= *[0-9.]*' | grep -o '[0-9.]*')
    echo "round $r | $v | wall ${wall} s | loop ${loop} s | HIP up at ${up} ms | pipelines set up at ${ps} ms | exit ${ex} ms" | tee -a "$OUT/summary.txt"
  done
done
ref=$OUT/results_1_1.cand
for f in "$OUT"/results_*.cand; do cmp -s "$ref" "$f" || echo "DIFFERS: $f"; done
echo "results compared (date line aside)"
