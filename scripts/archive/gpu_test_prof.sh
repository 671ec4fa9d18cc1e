set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -q -m gpu -x > gpurun_out/tests.log 2>&1 || { echo TEST_FAIL; tail -40 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --gpus 1 --steps 1 --warmup 1 --templates 400 > gpurun_out/prof.log 2>&1 || { echo PROF_FAIL; tail -30 gpurun_out/prof.log; exit 1; }
timeout -k 10 400 python bench.py --gpus 1 --steps 2 --warmup 1 > gpurun_out/bench1.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench1.log; exit 1; }
tail -1 gpurun_out/bench1.log
