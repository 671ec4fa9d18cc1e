# Round 3: re-check of the engine knobs after the direct-read harmonic sum
# (candidate list read in place, three batches in flight, 4 pipelines), then
# the app's phase timeline with process start-up / exit split off.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
EXPS="- BRP_FG=both BRP_INFLIGHT=3 - BRP_FG=both BRP_INFLIGHT=3" timeout -k 10 600 bash scripts/gpu_ab_bench.sh || exit $?
for st in 4 2 3; do
  timeout -k 10 200 python bench.py --steps 2 --warmup 1 --streams $st > gpurun_out/knob_streams.log 2>&1 || { echo FAIL streams $st; tail gpurun_out/knob_streams.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/knob_streams.log').read().strip().splitlines()[-1]); print('streams', sys.argv[1], d['value'], d.get('recall_vs_golden'))" $st
done
for i in 1 2 3; do
  BRP_PHASES=1 WORK=/tmp/appb timeout -k 10 120 bash scripts/bench_single.sh > gpurun_out/knob_app$i.log 2>&1 || { echo APP_FAIL; tail -20 /tmp/appb/app.log; exit 1; }
  cat gpurun_out/knob_app$i.log; grep "\[phase\]" /tmp/appb/app.log | cut -c1-60
done
