# A/B of pipelines sharing one series buffer (BRP_SHARE_SERIES=1, default) vs a
# device-to-device copy per pipeline (=0), then the GPU tests (run via gpurun).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/share
for sh in 0 1 0 1; do
  BRP_SHARE_SERIES=$sh timeout -k 10 200 python bench.py ${BENCH_ARGS:-} > gpurun_out/share/s$sh.log 2>&1 \
    || { echo BENCH_FAIL; tail -20 gpurun_out/share/s$sh.log; exit 1; }
  echo "share=$sh $(tail -1 gpurun_out/share/s$sh.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["recall_vs_golden"], d["table_identical_to_warmup"])')"
done
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread \
  > gpurun_out/share/tests.log 2>&1 || { echo TEST_FAIL; tail -40 gpurun_out/share/tests.log; exit 1; }
tail -1 gpurun_out/share/tests.log
