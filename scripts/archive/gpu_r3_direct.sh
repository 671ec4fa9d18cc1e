# Round 3: direct (unstaged) bound reads in the pruned harmonic sum
# (BRP_HS_DIRECT=1): bit-exactness tests, interleaved bench A/B (fp32 and
# config 5), kernel stats with the switch on.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k harmonic > gpurun_out/r3_direct_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r3_direct_tests.log; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|assert" gpurun_out/r3_direct_tests.log | head; exit $rc; }
EXPS="- BRP_HS_DIRECT=1 - BRP_HS_DIRECT=1 - BRP_HS_DIRECT=1" timeout -k 10 600 bash scripts/gpu_ab_bench.sh || exit $?
EXPS="- BRP_HS_DIRECT=1 - BRP_HS_DIRECT=1" BENCH_ARGS=--ps-fp16 timeout -k 10 400 bash scripts/gpu_ab_bench.sh || exit $?
rm -rf gpurun_out/prof_direct
BRP_HS_DIRECT=1 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_direct -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/prof_direct.log 2>&1 || { echo PROF_FAIL; tail gpurun_out/prof_direct.log; exit 1; }
python3 scripts/kstats.py gpurun_out/prof_direct/run_kernel_stats.csv > gpurun_out/prof_direct_stats.txt; head -8 gpurun_out/prof_direct_stats.txt
