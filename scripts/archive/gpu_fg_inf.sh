# With two batches in flight: graph replay (default) vs direct launches
# (BRP_NO_GRAPH=1), with and without the candidate list read in place
# (BRP_FG=both, no copyBuffer per batch), interleaved in one call.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2 3; do
  for e in "X=0" "BRP_NO_GRAPH=1" "BRP_NO_GRAPH=1 BRP_FG=both"; do
    env $e timeout -k 10 200 python bench.py --steps 4 --warmup 1 > gpurun_out/bench_fgi.log 2>&1 || { echo "BENCH FAIL $e"; tail -20 gpurun_out/bench_fgi.log; exit 1; }
    echo "bench $e $(python -c "import json,sys; d=json.loads(open('gpurun_out/bench_fgi.log').read().strip().splitlines()[-1]); print(d['value'], d['recall_vs_golden']['table'], d['table_identical_to_warmup'])")"
  done
done
