# per-stage timings (stagebench, batch 8) + rocprofv3 kernel stats of an 800-template bench
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
timeout -k 10 200 python tools/stagebench.py 8 > gpurun_out/stage.log 2>&1 || { echo STAGE_FAIL; tail -30 gpurun_out/stage.log; exit 1; }
tail -1 gpurun_out/stage.log
rm -rf gpurun_out/prof/*
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --gpus 1 --steps 1 --warmup 1 --templates 800 > gpurun_out/prof.log 2>&1 || { echo PROF_FAIL; tail -30 gpurun_out/prof.log; exit 1; }
python3 scripts/kstats.py $(find gpurun_out/prof -name '*kernel_stats.csv' | head -1)
