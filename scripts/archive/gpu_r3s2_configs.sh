# Round 3 session 2: configs 4 and 5 at the new defaults, and the BOINC app on the reference
# protocol (whole process, phase timeline), result file checked against the golden file.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --ps-fp16 --steps 3 --warmup 1 > gpurun_out/cfg5.log 2>&1 || { echo CFG5_FAIL; tail -20 gpurun_out/cfg5.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/cfg5.log').read().strip().splitlines()[-1]); print('cfg5', d['value'], d['ms_per_step'], d['recall_vs_golden'])"
timeout -k 10 600 python bench.py --wus 8 --steps 1 --warmup 1 > gpurun_out/cfg4.log 2>&1 || { echo CFG4_FAIL; tail -20 gpurun_out/cfg4.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/cfg4.log').read().strip().splitlines()[-1]); print('cfg4', d['value'], d['ms_per_step'], d['recall_vs_golden'])"
for i in 1 2 3; do
  BRP_PHASES=1 WORK=/tmp/appb timeout -k 10 120 bash scripts/bench_single.sh > gpurun_out/app$i.log 2>&1 || { echo APP_FAIL; tail -20 /tmp/appb/app.log; exit 1; }
  cat gpurun_out/app$i.log; grep "\[phase\]" /tmp/appb/app.log > gpurun_out/app_phases$i.log
done
python3 - <<'PY'
import sys
sys.path.insert(0, ".")
from boinc_app_eah_brp_amd import native
brp = native()
got, done = brp.read_results("/tmp/appb/results.cand")
ref, _ = brp.read_results("data/golden/bench_wu_cpu_results.txt")
print("app result lines", len(got), "golden", len(ref), "done", done,
      "identical" if [tuple(x) for x in got] == [tuple(x) for x in ref] else "DIFFER")
PY
