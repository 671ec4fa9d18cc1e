# Per-kernel times of the pruned harmonic sum (stage benchmark, batch 1), at the
# chi^2 thresholds and with no exact work (BRP_STAGE_THR_SCALE=1000).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for sc in 1 1000; do
  rm -rf gpurun_out/hspprof$sc; mkdir -p gpurun_out/hspprof$sc
  BRP_STAGE_THR_SCALE=$sc timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/hspprof$sc -o run --output-format csv -- python3 tools/stagebench.py 1 > gpurun_out/hspprof$sc/log.txt 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/hspprof$sc/log.txt; exit 1; }
  echo "scale $sc: $(tail -1 gpurun_out/hspprof$sc/log.txt)"
  python3 scripts/kstats.py gpurun_out/hspprof$sc/run_kernel_stats.csv | head -8
done
