#!/bin/bash
# Whole-process time on the reference protocol (scripts/bench_single.sh), round 6:
# N runs of the application with BRP_PHASES=1 (phase times + the process start /
# exit around them), the result files compared byte for byte, then one run under
# rocprofv3 --hip-trace --kernel-trace (HIP API calls of the start-up; BRP_FAST_EXIT=0
# so that the profiler can write its output at exit).
# Usage (GPU box): scripts/gpu_r6_startup.sh [runs] [outdir]   (APP= another binary)
set -uo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
N=${1:-3}
OUT=${2:-$ROOT/gpurun_out/r6_startup}
mkdir -p "$OUT" && OUT=$(cd "$OUT" && pwd)
APP=${APP:-$ROOT/bin/einsteinbinary_mi355x}
mkdir -p "$OUT"
export TMPDIR=/tmp
for i in $(seq 1 "$N"); do
  W=/tmp/r6_bs_$i
  rm -rf "$W"
  BRP_PHASES=1 WORK=$W APP=$APP timeout -k 10 120 "$ROOT/scripts/bench_single.sh" > "$OUT/run_$i.txt" 2>&1 || { echo "run $i failed"; cat "$OUT/run_$i.txt"; exit 1; }
  grep '\[phase\]' "$W/app.log" | sed 's/  epoch_ms=.*//' >> "$OUT/run_$i.txt"
  cp "$W/results.cand" "$OUT/results_$i.cand"
  cat "$OUT/run_$i.txt"
done
# the result files differ only in the header's date line
for i in $(seq 2 "$N"); do
  if cmp <(grep -v '^% Date:' "$OUT/results_1.cand") <(grep -v '^% Date:' "$OUT/results_$i.cand"); then
    echo "results_$i.cand identical to results_1.cand (date line aside)"
  fi
done
if [ "${TRACE:-1}" = "1" ]; then
  W=/tmp/r6_bs_trace
  rm -rf "$W" && mkdir -p "$W" && cd "$W"
  D=$ROOT/data/testwu
  BRP_FAST_EXIT=0 timeout -k 10 120 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d "$OUT/trace" -o app -- \
    "$APP" -i "$D/p2030.20151015.G187.41-00.88.N.b2s0g0.00000_1099.bin4" -t "$D/stochastic_full.bank" \
    -l "$D/p2030.20151015.G187.41-00.88.N.b2s0g0.00000.zap" -o results.cand -c checkpoint.cpt -A 0.08 -P 3.0 -f 400.0 -W \
    > "$OUT/trace_app.log" 2>&1 || { echo "trace run failed"; tail -20 "$OUT/trace_app.log"; exit 1; }
fi
echo done
