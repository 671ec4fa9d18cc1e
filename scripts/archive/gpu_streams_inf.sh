# Pipelines per GPU and device batch with two batches in flight per pipeline,
# interleaved in one call.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do
  for cfg in "--streams 3 --batch 1" "--streams 2 --batch 1" "--streams 4 --batch 1" "--streams 2 --batch 2"; do
    timeout -k 10 200 python bench.py --steps 4 --warmup 1 $cfg > gpurun_out/bench_si.log 2>&1 || { echo "BENCH FAIL $cfg"; tail -20 gpurun_out/bench_si.log; exit 1; }
    echo "bench $cfg $(python -c "import json,sys; d=json.loads(open('gpurun_out/bench_si.log').read().strip().splitlines()[-1]); print(d['value'], d['recall_vs_golden']['table'], d['table_identical_to_warmup'])")"
  done
done
