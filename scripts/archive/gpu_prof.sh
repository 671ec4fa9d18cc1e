set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --gpus 1 --steps 1 --warmup 1 --templates 400 > gpurun_out/prof.log 2>&1 || { echo PROF_FAIL; tail -30 gpurun_out/prof.log; exit 1; }
tail -2 gpurun_out/prof.log
find gpurun_out/prof -name "*stats*" | head
