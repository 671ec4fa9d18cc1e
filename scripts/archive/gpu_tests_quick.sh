# Selected GPU tests (pytest -k expression in $K) under the usual per-test timeouts.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread -k "${K:-gpu}" \
  > gpurun_out/quick_tests.log 2>&1 || { echo TEST_FAIL; tail -60 gpurun_out/quick_tests.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/quick_tests.log | tail -15
