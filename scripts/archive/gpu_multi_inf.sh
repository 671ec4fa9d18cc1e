# Multi-WU batching and config 5 with two batches in flight: GPU search tests,
# then config 4 (8 WUs) and config 5 benches against BRP_INFLIGHT=1 in one call.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_search.py -x -v -m gpu --timeout 120 --timeout-method thread \
  > gpurun_out/mi_tests.log 2>&1 || { echo TEST_FAIL; tail -60 gpurun_out/mi_tests.log; exit 1; }
tail -2 gpurun_out/mi_tests.log
for cfg in "--wus 8" "--ps-fp16"; do
  for e in BRP_INFLIGHT=1 BRP_INFLIGHT=2; do
    env $e timeout -k 10 300 python bench.py --steps 2 --warmup 1 $cfg > gpurun_out/bench_mi.log 2>&1 || { echo "BENCH FAIL $cfg $e"; tail -20 gpurun_out/bench_mi.log; exit 1; }
    echo "bench $cfg $e $(python -c "import json,sys; d=json.loads(open('gpurun_out/bench_mi.log').read().strip().splitlines()[-1]); print(d['value'], d['recall_vs_golden'], d['table_identical_to_warmup'])")"
  done
done
