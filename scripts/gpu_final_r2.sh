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
