# Rehearsal of the driver's round-end GPU tiers (run via gpurun):
# pytest -m gpu, smoke(), then the default 1-GPU bench.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread \
  > gpurun_out/re_tests.log 2>&1 || { echo TEST_FAIL; tail -60 gpurun_out/re_tests.log; exit 1; }
tail -2 gpurun_out/re_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/re_smoke.log 2>&1 \
  || { echo SMOKE_FAIL; tail -30 gpurun_out/re_smoke.log; exit 1; }
tail -1 gpurun_out/re_smoke.log
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > gpurun_out/re_bench.log 2>&1 \
  || { echo BENCH_FAIL; tail -30 gpurun_out/re_bench.log; exit 1; }
tail -1 gpurun_out/re_bench.log
