# isolated per-kernel times (one pipeline, no kernel overlap) of the chirp-z
# path: rocprofv3 kernel trace of bench.py --streams 1 at the given paddings
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for P in ${PADDINGS:-2.7 2.9}; do
  rm -rf gpurun_out/iso_$P; mkdir -p gpurun_out/iso_$P
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/iso_$P -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --padding $P --streams 1 --templates ${TEMPLATES:-300} ${BENCH_ARGS:-} > gpurun_out/iso_$P.log 2>&1 || { echo PROF_FAIL $P; tail -30 gpurun_out/iso_$P.log; exit 1; }
  python3 scripts/kstats.py $(find gpurun_out/iso_$P -name '*kernel_stats.csv' | head -1) > gpurun_out/kstats_iso_$P.txt
  echo "== P $P"; head -12 gpurun_out/kstats_iso_$P.txt
done
