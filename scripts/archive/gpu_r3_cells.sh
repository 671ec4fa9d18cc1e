# Round 3: pass-3 row-order cells + transpose instead of hs_cells_kernel
# (BRP_P3_CELLS): tests, interleaved bench A/B (fp32, config 5), kernel stats.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PYT="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_gpu_kernels.py > gpurun_out/r3_cells_kernels.log 2>&1
rc=$?; tail -1 gpurun_out/r3_cells_kernels.log; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/r3_cells_kernels.log | head -20; exit $rc; }
timeout -k 10 600 $PYT tests/test_gpu_search.py tests/test_gpu_headline.py > gpurun_out/r3_cells_search.log 2>&1
rc=$?; tail -1 gpurun_out/r3_cells_search.log; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/r3_cells_search.log | head -20; exit $rc; }
EXPS="- BRP_P3_CELLS=0 - BRP_P3_CELLS=0 - BRP_P3_CELLS=0" timeout -k 10 600 bash scripts/gpu_ab_bench.sh || exit $?
EXPS="- BRP_P3_CELLS=0 - BRP_P3_CELLS=0" BENCH_ARGS=--ps-fp16 timeout -k 10 400 bash scripts/gpu_ab_bench.sh || exit $?
rm -rf gpurun_out/prof_cells
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cells -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/prof_cells.log 2>&1 || { echo PROF_FAIL; tail gpurun_out/prof_cells.log; exit 1; }
python3 scripts/kstats.py gpurun_out/prof_cells/run_kernel_stats.csv > gpurun_out/prof_cells_stats.txt; head -9 gpurun_out/prof_cells_stats.txt
