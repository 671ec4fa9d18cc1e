# rocprofv3 kernel trace + stats of the bench (default batch/pipelines), summary -> gpurun_out/prof
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/prof; mkdir -p gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --gpus 1 --steps 1 --warmup 1 ${BENCH_ARGS:-} > gpurun_out/prof.log 2>&1 || { echo PROF_FAIL; tail -30 gpurun_out/prof.log; exit 1; }
tail -1 gpurun_out/prof.log
python3 scripts/kstats.py $(find gpurun_out/prof -name '*kernel_stats.csv' | head -1)
