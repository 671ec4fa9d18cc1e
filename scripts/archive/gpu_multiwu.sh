set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/tests_all.log 2>&1 || { echo TEST_FAIL; tail -60 gpurun_out/tests_all.log; exit 1; }
tail -1 gpurun_out/tests_all.log
timeout -k 10 600 python bench.py --steps 1 --warmup 1 --wus ${WUS:-8} --templates ${TPL:-0} > gpurun_out/bench_wus.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/bench_wus.log; exit 1; }
tail -1 gpurun_out/bench_wus.log
