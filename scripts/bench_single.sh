#!/bin/bash
# The reference benchmark protocol (debian/extra/einstein_bench/bench_single.sh:28)
# on the MI355X application: the shipped 2^22-sample WU against the full
# stochastic_full.bank with -A 0.08 -P 3.0 -f 400.0 -W, wall-clock timed.
# Usage: scripts/bench_single.sh [extra app options, e.g. -z or -D 1]
# Env: APP (binary), WORK (scratch dir, default: a new temp dir)
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
APP=${APP:-$ROOT/bin/einsteinbinary_mi355x}
D=$ROOT/data/testwu
WU=$D/p2030.20151015.G187.41-00.88.N.b2s0g0.00000_1099.bin4
ZAP=$D/p2030.20151015.G187.41-00.88.N.b2s0g0.00000.zap
BANK=$D/stochastic_full.bank
WORK=${WORK:-$(mktemp -d)}
mkdir -p "$WORK"
cd "$WORK"
rm -f results.cand checkpoint.cpt
t0=$(date +%s.%N)
"$APP" -i "$WU" -t "$BANK" -l "$ZAP" -o results.cand -c checkpoint.cpt -A 0.08 -P 3.0 -f 400.0 -W "$@" 2> app.log
t1=$(date +%s.%N)
n=$(grep -c . "$BANK")
python3 - "$t0" "$t1" "$n" <<'PY'
import sys
t0, t1, n = float(sys.argv[1]), float(sys.argv[2]), int(sys.argv[3])
print(f"bench_single: {n} templates in {t1 - t0:.3f} s wall (process incl. start-up, WU read, whitening): {n / (t1 - t0):.1f} templates/s")
PY
grep "Throughput" app.log || true
if grep -q "epoch_ms=" app.log; then  # BRP_PHASES=1: process start-up and exit around the phases
  python3 - "$t0" "$t1" app.log <<'PY'
import re, sys
t0, t1 = float(sys.argv[1]) * 1e3, float(sys.argv[2]) * 1e3
ph = [(m.group(1).strip(), float(m.group(2)), float(m.group(3))) for m in
      re.finditer(r"\[phase\] (.*?) t=\s*([\d.]+) ms .*epoch_ms=([\d.]+)", open(sys.argv[3]).read())]
first_t, first_e = ph[0][1], ph[0][2]
static_init = first_e - first_t  # wall time of the phase clock's zero (static initialisation)
print(f"process: exec + loading to static init {static_init - t0:.1f} ms; last phase '{ph[-1][0]}' to exit {t1 - ph[-1][2]:.1f} ms")
PY
fi
