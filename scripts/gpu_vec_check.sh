# packed-math A/B: GPU tests of the FFT paths, then interleaved bench A/B (head vs ab/old)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1200 python -u -m pytest ${TESTS:-tests/test_gpu_headline.py tests/test_gpu_kernels.py tests/test_gpu_search.py tests/test_gpu_radix7.py} -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/vec_tests.log 2>&1 || { echo TEST_FAIL; tail -60 gpurun_out/vec_tests.log; exit 1; }
tail -1 gpurun_out/vec_tests.log
ROUNDS=3 STEPS=2 BENCH_ARGS="" bash scripts/gpu_ab_so.sh
ROUNDS=1 STEPS=1 BENCH_ARGS="--padding 2.7" bash scripts/gpu_ab_so.sh
