# Full GPU test suite + per-stage timings (run via gpurun)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu -x > gpurun_out/tests_all.log 2>&1 || { echo TEST_FAIL; tail -60 gpurun_out/tests_all.log; exit 1; }
tail -3 gpurun_out/tests_all.log
timeout -k 10 300 python tools/stagebench.py 4 > gpurun_out/stage.log 2>&1 || { echo STAGE_FAIL; tail -30 gpurun_out/stage.log; exit 1; }
tail -1 gpurun_out/stage.log
