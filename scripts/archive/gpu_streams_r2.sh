# Pipelines per GPU (3 / 4 / 5) and graph vs direct launches after the pruned
# harmonic sum (GPU busy fraction fell to 94 %), interleaved in one call.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do
  for cfg in "X=0 --streams 3" "X=0 --streams 4" "X=0 --streams 5" "BRP_NO_GRAPH=1 --streams 3"; do
    set -- $cfg
    env $1 timeout -k 10 200 python bench.py --steps 4 --warmup 1 $2 $3 > gpurun_out/bench_str.log 2>&1 || { echo "BENCH FAIL $cfg"; tail -20 gpurun_out/bench_str.log; exit 1; }
    echo "bench $cfg $(python -c "import json,sys; d=json.loads(open('gpurun_out/bench_str.log').read().strip().splitlines()[-1]); print(d['value'], d['recall_vs_golden']['table'], d['table_identical_to_warmup'])")"
  done
done
