# Re-check of the pass-2 persistent workgroups per CU and of 4 pipelines at the
# new defaults (two batches in flight, direct launches), interleaved in one call.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v -m gpu --timeout 120 --timeout-method thread \
  -k "in_flight or harmonic_sum_bench" > gpurun_out/pr_tests.log 2>&1 || { echo TEST_FAIL; tail -60 gpurun_out/pr_tests.log; exit 1; }
tail -2 gpurun_out/pr_tests.log
for r in 1 2; do
  for cfg in "X=0 --streams 3" "BRP_PERSIST=0 --streams 3" "BRP_PERSIST=6 --streams 3" "BRP_PERSIST=3 --streams 3" "X=0 --streams 4"; do
    set -- $cfg
    env $1 timeout -k 10 200 python bench.py --steps 4 --warmup 1 $2 $3 > gpurun_out/bench_pr.log 2>&1 || { echo "BENCH FAIL $cfg"; tail -20 gpurun_out/bench_pr.log; exit 1; }
    echo "bench $cfg $(python -c "import json,sys; d=json.loads(open('gpurun_out/bench_pr.log').read().strip().splitlines()[-1]); print(d['value'], d['recall_vs_golden']['table'], d['table_identical_to_warmup'])")"
  done
done
