# Wide-window device running median: exactness tests and timing at the
# benchmark spectrum size for several windows.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -v -m gpu --timeout 200 --timeout-method thread -k "running_median or whitening" \
  > gpurun_out/rmed_tests.log 2>&1 || { echo TEST_FAIL; tail -60 gpurun_out/rmed_tests.log; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/rmed_tests.log | tail -20
timeout -k 10 300 python tools/rmed_bench.py 1000 3072 3073 10000 12288 12289 30000 100000 250000 > gpurun_out/rmed_bench.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/rmed_bench.log; exit 1; }
cat gpurun_out/rmed_bench.log
