#!/bin/bash
# Concurrent-instance benchmark after debian/extra/einstein_bench/runall.sh:12-25:
# N copies of the application run at once (instance k on GPU k % GPUS, each in
# its own directory like a BOINC slot), progress is polled from each slot's
# graphics shared memory file boinc_EinsteinRadio_0 (<fraction_done>), and the
# aggregate templates/s of the node is printed at the end.
# Usage: scripts/runall.sh N [GPUS]
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
N=${1:-2}
GPUS=${2:-1}
APP=${APP:-$ROOT/bin/einsteinbinary_mi355x}
D=$ROOT/data/testwu
WU=$D/p2030.20151015.G187.41-00.88.N.b2s0g0.00000_1099.bin4
ZAP=$D/p2030.20151015.G187.41-00.88.N.b2s0g0.00000.zap
BANK=$D/stochastic_full.bank
WORK=${WORK:-$(mktemp -d)}
pids=()
t0=$(date +%s.%N)
for k in $(seq 0 $((N - 1))); do
  mkdir -p "$WORK/slot$k"
  (cd "$WORK/slot$k" && rm -f results.cand checkpoint.cpt &&
   exec "$APP" -i "$WU" -t "$BANK" -l "$ZAP" -o results.cand -c checkpoint.cpt -A 0.08 -P 3.0 -f 400.0 -W \
        -D $((k % GPUS)) 2> app.log) &
  pids+=($!)
done
running=1
while [ $running -eq 1 ]; do
  sleep 1
  running=0
  line=""
  for k in $(seq 0 $((N - 1))); do
    kill -0 "${pids[$k]}" 2>/dev/null && running=1
    f=$(tr -d '\0' < "$WORK/slot$k/boinc_EinsteinRadio_0" 2>/dev/null | sed -n 's:.*<fraction_done>\(.*\)</fraction_done>.*:\1:p' || true)
    line="$line slot$k=${f:-?}"
  done
  echo "progress:$line"
done
rc=0
for p in "${pids[@]}"; do wait "$p" || rc=1; done
t1=$(date +%s.%N)
n=$(grep -c . "$BANK")
python3 - "$t0" "$t1" "$n" "$N" <<'PY'
import sys
t0, t1, n, k = float(sys.argv[1]), float(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
print(f"runall: {k} instances x {n} templates in {t1 - t0:.3f} s: {k * n / (t1 - t0):.1f} templates/s aggregate")
PY
exit $rc
