# Config 5 (fp16 spectrum) through the pruned harmonic sum: tests, then bench
# A/B (pruned vs full gather on the fp16 spectrum, and the fp32 default) in one call.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_search.py -x -v -m gpu --timeout 120 \
  --timeout-method thread -k "harmonic or fp16" > gpurun_out/hs16_tests.log 2>&1 || { echo TEST_FAIL; tail -60 gpurun_out/hs16_tests.log; exit 1; }
tail -2 gpurun_out/hs16_tests.log
for r in 1 2; do
  for e in "BRP_HS_FULL=1 --ps-fp16" "BRP_HS_FULL=0 --ps-fp16" "BRP_HS_FULL=0"; do
    set -- $e
    env $1 timeout -k 10 200 python bench.py --steps 4 --warmup 1 $2 > gpurun_out/bench_hs16.log 2>&1 || { echo "BENCH FAIL $e"; tail -20 gpurun_out/bench_hs16.log; exit 1; }
    echo "bench $e $(python -c "import json,sys; d=json.loads(open('gpurun_out/bench_hs16.log').read().strip().splitlines()[-1]); print(d['value'], d['recall_vs_golden'], d['table_identical_to_warmup'])")"
  done
done
