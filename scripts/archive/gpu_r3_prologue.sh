# Round 3: pass-1 / pass-3 prologue loads issued in one round (head) vs ab/prev:
# kernel + search tests, interleaved A/B (fp32 3 rounds, config 5 2 rounds).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PYT="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_gpu_kernels.py tests/test_gpu_headline.py tests/test_gpu_bluestein.py > gpurun_out/r3_pro_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r3_pro_tests.log; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|assert" gpurun_out/r3_pro_tests.log | head; exit $rc; }
ROUNDS=3 timeout -k 10 600 bash scripts/gpu_ab_so.sh > gpurun_out/r3_pro_ab.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/r3_pro_ab.log; exit 1; }
grep round gpurun_out/r3_pro_ab.log
ROUNDS=2 BENCH_ARGS=--ps-fp16 timeout -k 10 600 bash scripts/gpu_ab_so.sh > gpurun_out/r3_pro_ab16.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/r3_pro_ab16.log; exit 1; }
grep round gpurun_out/r3_pro_ab16.log
