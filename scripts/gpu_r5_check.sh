# round-5 checks: stride probe, radix-7 and bounded-output GPU tests
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 ./build/probe/stride_probe > gpurun_out/stride_probe.txt 2>&1 || { echo PROBE_FAIL; cat gpurun_out/stride_probe.txt; exit 1; }
cat gpurun_out/stride_probe.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_radix7.py tests/test_gpu_bounded.py -x -v -m gpu --timeout 150 --timeout-method thread > gpurun_out/r5_tests.log 2>&1 || { echo TEST_FAIL; tail -60 gpurun_out/r5_tests.log; exit 1; }
tail -15 gpurun_out/r5_tests.log
