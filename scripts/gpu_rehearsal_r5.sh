# round-end rehearsal + bench kernel profile (outputs under gpurun_out/)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash scripts/gpu_roundend.sh || exit 1
BENCH_ARGS="" bash scripts/gpu_profile.sh > gpurun_out/prof_bench_summary.txt 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/prof_bench_summary.txt; exit 1; }
head -12 gpurun_out/prof_bench_summary.txt
