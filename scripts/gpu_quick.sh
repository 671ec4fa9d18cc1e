# GPU kernel tests + stage timings + pass-3 ablations (quick iteration loop)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/tests_all.log 2>&1 || { echo TEST_FAIL; tail -60 gpurun_out/tests_all.log; exit 1; }
tail -1 gpurun_out/tests_all.log
for e in ${P3EXPS:-0}; do
  BRP_P3_EXP=$e timeout -k 10 120 python tools/stagebench.py 4 > gpurun_out/p3exp_$e.log 2>&1 || { echo FAIL $e; tail -20 gpurun_out/p3exp_$e.log; exit 1; }
  echo "exp=$e $(tail -1 gpurun_out/p3exp_$e.log)"
done
