set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
tail -3 gpurun_out/smoke.log
timeout -k 10 400 python bench.py --gpus 1 --steps 2 --warmup 1 > gpurun_out/bench1.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench1.log; exit 1; }
tail -3 gpurun_out/bench1.log
