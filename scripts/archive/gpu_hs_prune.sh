# Pruned harmonic sum: bit-exactness tests, then stage timings and bench A/B
# against the full gather kernel (BRP_HS_FULL=1), interleaved in one call.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -v -m gpu --timeout 120 --timeout-method thread \
  -k "harmonic" > gpurun_out/hsp_tests.log 2>&1 || { echo TEST_FAIL; tail -60 gpurun_out/hsp_tests.log; exit 1; }
tail -2 gpurun_out/hsp_tests.log
for e in BRP_HS_FULL=1 BRP_HS_FULL=0; do
  env $e timeout -k 10 120 python tools/stagebench.py 1 > gpurun_out/stage_hsp.log 2>&1 || { echo "FAIL $e"; tail -20 gpurun_out/stage_hsp.log; exit 1; }
  echo "stage $e $(tail -1 gpurun_out/stage_hsp.log)"
done
for r in 1 2; do
  for e in BRP_HS_FULL=1 BRP_HS_FULL=0; do
    env $e timeout -k 10 200 python bench.py --steps 4 --warmup 1 > gpurun_out/bench_hsp.log 2>&1 || { echo "BENCH FAIL $e"; tail -20 gpurun_out/bench_hsp.log; exit 1; }
    echo "bench $e $(python -c "import json,sys; d=json.loads(open('gpurun_out/bench_hsp.log').read().strip().splitlines()[-1]); print(d['value'], d['recall_vs_golden'], d['table_identical_to_warmup'])")"
  done
done
