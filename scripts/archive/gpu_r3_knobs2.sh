# Round 3: env knobs re-checked at the current head: pruned HS blocks
# XCD-contiguous (BRP_HS_XCD=1), candidate list read in place (BRP_FG=both).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 env BRP_HS_XCD=1 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "bench_size" > gpurun_out/r3_k2_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r3_k2_tests.log; [ $rc -eq 0 ] || exit $rc
EXPS="- BRP_HS_XCD=1 BRP_FG=both - BRP_HS_XCD=1 BRP_FG=both - BRP_HS_XCD=1 BRP_FG=both" timeout -k 10 900 bash scripts/gpu_ab_bench.sh || exit $?
