# Round 3: direct bound reads with all 16 loads in flight at once (head) vs
# the loads issued in pairs (ab/prev): HS tests, interleaved A/B, config 5.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "harmonic or cells" > gpurun_out/r3_hsload_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r3_hsload_tests.log; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|assert" gpurun_out/r3_hsload_tests.log | head; exit $rc; }
ROUNDS=3 timeout -k 10 600 bash scripts/gpu_ab_so.sh > gpurun_out/r3_hsload_ab.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/r3_hsload_ab.log; exit 1; }
grep round gpurun_out/r3_hsload_ab.log
ROUNDS=2 BENCH_ARGS=--ps-fp16 timeout -k 10 600 bash scripts/gpu_ab_so.sh > gpurun_out/r3_hsload_ab16.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/r3_hsload_ab16.log; exit 1; }
grep round gpurun_out/r3_hsload_ab16.log
