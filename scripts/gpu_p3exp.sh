# pass-3 ablations via BRP_P3_EXP (stage timings)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for e in 0 1 2 3 4 8 12; do
  BRP_P3_EXP=$e timeout -k 10 120 python tools/stagebench.py 4 > gpurun_out/p3exp_$e.log 2>&1 || { echo FAIL $e; tail -20 gpurun_out/p3exp_$e.log; exit 1; }
  echo "exp=$e $(tail -1 gpurun_out/p3exp_$e.log)"
done
