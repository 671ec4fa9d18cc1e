set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --steps 5 --warmup 1 > gpurun_out/base_b1.log 2>&1 || { echo B1FAIL; tail -20 gpurun_out/base_b1.log; exit 1; }
tail -1 gpurun_out/base_b1.log
for P in 3.5 2.7 2.9 1.1; do
timeout -k 10 200 python bench.py --steps 1 --warmup 1 --padding $P > gpurun_out/base_p$P.log 2>&1 || { echo PFAIL $P; tail -20 gpurun_out/base_p$P.log; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/base_p$P.log $P
done
rm -rf gpurun_out/prof27; mkdir -p gpurun_out/prof27
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof27 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --padding 2.7 > gpurun_out/prof27.log 2>&1 || { echo PROF_FAIL; tail -30 gpurun_out/prof27.log; exit 1; }
python3 scripts/kstats.py $(find gpurun_out/prof27 -name '*kernel_stats.csv' | head -1) > gpurun_out/kstats_p27.txt
head -30 gpurun_out/kstats_p27.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_rccl.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/base_rccl.log 2>&1 || { echo RCCL_FAIL; tail -40 gpurun_out/base_rccl.log; exit 1; }
tail -3 gpurun_out/base_rccl.log
