set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/tests_all.log 2>&1 || { echo TEST_FAIL; tail -60 gpurun_out/tests_all.log; exit 1; }
tail -1 gpurun_out/tests_all.log
for p in ${PERSISTS:-0 4 6 8}; do
  BRP_PERSIST=$p timeout -k 10 120 python tools/stagebench.py 4 > gpurun_out/persist_$p.log 2>&1 || { echo FAIL $p; tail -20 gpurun_out/persist_$p.log; exit 1; }
  echo "persist=$p $(tail -1 gpurun_out/persist_$p.log)"
done
