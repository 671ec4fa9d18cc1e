# Two batches in flight per pipeline (submit / complete) vs one: GPU tests,
# bench A/B interleaved in one call, then kernel trace busy fraction.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread \
  > gpurun_out/inf_tests.log 2>&1 || { echo TEST_FAIL; tail -60 gpurun_out/inf_tests.log; exit 1; }
tail -2 gpurun_out/inf_tests.log
for r in 1 2; do
  for e in BRP_INFLIGHT=1 BRP_INFLIGHT=2; do
    env $e timeout -k 10 200 python bench.py --steps 4 --warmup 1 > gpurun_out/bench_inf.log 2>&1 || { echo "BENCH FAIL $e"; tail -20 gpurun_out/bench_inf.log; exit 1; }
    echo "bench $e $(python -c "import json,sys; d=json.loads(open('gpurun_out/bench_inf.log').read().strip().splitlines()[-1]); print(d['value'], d['recall_vs_golden'], d['table_identical_to_warmup'])")"
  done
done
bash scripts/gpu_profile.sh > gpurun_out/inf_prof.txt 2>&1 || { echo PROF_FAIL; tail gpurun_out/inf_prof.txt; exit 1; }
python3 scripts/trace_busy.py gpurun_out/prof/run_kernel_trace.csv | head -3
