# Round-end rehearsal plus config 5 and a fresh per-kernel profile (run via gpurun).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/final
bash scripts/gpu_roundend.sh || exit 1
timeout -k 10 200 python bench.py --ps-fp16 > gpurun_out/final/fp16.log 2>&1 || { echo FP16_FAIL; tail -20 gpurun_out/final/fp16.log; exit 1; }
tail -1 gpurun_out/final/fp16.log
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final/prof -o run -- \
  python3 bench.py --steps 1 --warmup 1 > gpurun_out/final/prof.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/final/prof.log; exit 1; }
tail -1 gpurun_out/final/prof.log
