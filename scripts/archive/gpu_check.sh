# Round health check: GPU tests, smoke, 1-GPU bench (run via gpurun)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests_gpu.log 2>&1 || { echo TEST_FAIL; tail -60 gpurun_out/tests_gpu.log; exit 1; }
tail -3 gpurun_out/tests_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench1.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench1.log; exit 1; }
tail -4 gpurun_out/bench1.log
