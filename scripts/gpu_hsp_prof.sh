# Per-kernel times of the pruned harmonic sum (stage benchmark, batch 1).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/hspprof; mkdir -p gpurun_out/hspprof
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/hspprof -o run --output-format csv -- python3 tools/stagebench.py 1 > gpurun_out/hspprof/log.txt 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/hspprof/log.txt; exit 1; }
tail -1 gpurun_out/hspprof/log.txt
python3 scripts/kstats.py gpurun_out/hspprof/run_kernel_stats.csv | head -20
