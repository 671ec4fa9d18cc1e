# Round-end rehearsal at the new defaults (direct launches, two batches in
# flight), kernel stats, and config 5.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
bash scripts/gpu_roundend.sh || exit 1
bash scripts/gpu_profile.sh > gpurun_out/fin_prof.txt 2>&1 || { echo PROF_FAIL; tail gpurun_out/fin_prof.txt; exit 1; }
python3 scripts/trace_busy.py gpurun_out/prof/run_kernel_trace.csv | head -3
timeout -k 10 300 python bench.py --ps-fp16 > gpurun_out/fin_cfg5.log 2>&1 || { echo CFG5_FAIL; tail gpurun_out/fin_cfg5.log; exit 1; }
tail -1 gpurun_out/fin_cfg5.log | cut -c1-200
for r in 1 2; do
  for e in BRP_INFLIGHT=2 BRP_INFLIGHT=3; do
    env $e timeout -k 10 200 python bench.py --steps 4 --warmup 1 > gpurun_out/bench_d3.log 2>&1 || { echo "BENCH FAIL $e"; tail -20 gpurun_out/bench_d3.log; exit 1; }
    echo "bench $e $(python -c "import json,sys; d=json.loads(open('gpurun_out/bench_d3.log').read().strip().splitlines()[-1]); print(d['value'], d['recall_vs_golden']['table'], d['table_identical_to_warmup'])")"
  done
done
