# Register pass 3 (L3 = 256): numerics tests, then stage timings and bench A/B
# against the LDS-staged pass 3 (BRP_P3R=0), interleaved in one call.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_search.py -x -v -m gpu --timeout 120 --timeout-method thread \
  -k "register_kernel or fft_plans or bench_wu_prefix" > gpurun_out/p3r_tests.log 2>&1 \
  || { echo TEST_FAIL; tail -60 gpurun_out/p3r_tests.log; exit 1; }
tail -2 gpurun_out/p3r_tests.log
for e in BRP_P3R=0 BRP_P3R=8 BRP_P3R=4 BRP_P3R=108 BRP_P3R=104; do
  env ${e//,/ } timeout -k 10 120 python tools/stagebench.py 1 > gpurun_out/stage_p3r.log 2>&1 || { echo "FAIL $e"; tail -20 gpurun_out/stage_p3r.log; exit 1; }
  echo "stage $e $(tail -1 gpurun_out/stage_p3r.log)"
done
for r in 1 2; do
  for e in BRP_P3R=0 BRP_P3R=8 BRP_P3R=108 BRP_P3R=104; do
    env $e timeout -k 10 200 python bench.py --steps 4 --warmup 1 > gpurun_out/bench_p3r.log 2>&1 || { echo "BENCH FAIL $e"; tail -20 gpurun_out/bench_p3r.log; exit 1; }
    echo "bench $e $(python -c "import json,sys; d=json.loads(open('gpurun_out/bench_p3r.log').read().strip().splitlines()[-1]); print(d['value'], d['recall_vs_golden'])")"
  done
done
