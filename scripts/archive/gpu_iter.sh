# Iteration loop: GPU kernel tests, then stage timings under each env setting in $EXPS
# (space-separated, e.g. EXPS="BRP_PERSIST=6 BRP_SHARE_SERIES=0"; "-" = defaults)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_kernels.py} -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests_kern.log 2>&1 || { echo TEST_FAIL; tail -40 gpurun_out/tests_kern.log; exit 1; }
tail -1 gpurun_out/tests_kern.log
for e in ${EXPS:--}; do
  if [ "$e" = "-" ]; then envs=""; else envs="${e//,/ }"; fi
  env $envs timeout -k 10 120 python tools/stagebench.py ${BATCH:-8} > gpurun_out/stage_exp.log 2>&1 || { echo "FAIL $e"; tail -20 gpurun_out/stage_exp.log; exit 1; }
  echo "$e $(tail -1 gpurun_out/stage_exp.log)"
done
