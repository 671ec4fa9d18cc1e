# Round 3 GPU session: new kernels' tests, A/B bench against ab/*, PMC of the
# harmonic-sum / pass-3 LDS counters, the application's phase timeline.
# Test failures (pytest rc 1) are recorded and the script goes on; any other
# non-zero status (timeout, abort, crash) ends the script there.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
FAILED=""
step() {  # step <name> <timeout s> <command...>
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/r3_$name.log 2>&1
  local rc=$?
  if [ $rc -eq 0 ]; then echo "OK   $name  $(tail -1 gpurun_out/r3_$name.log)"; return 0; fi
  if [ $rc -eq 1 ]; then echo "FAIL $name"; grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/r3_$name.log | head -20; FAILED="$FAILED $name"; return 0; fi
  echo "ABORT $name rc=$rc"; tail -30 gpurun_out/r3_$name.log; exit $rc
}
PYT="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
step hs 300 $PYT tests/test_gpu_kernels.py -k "harmonic"
if [ -z "${SKIP_AB:-}" ]; then
  ROUNDS=${ROUNDS:-3} timeout -k 10 600 bash scripts/gpu_ab_so.sh > gpurun_out/r3_ab.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/r3_ab.log; exit 1; }
  grep round gpurun_out/r3_ab.log
fi
step kernels 400 $PYT tests/test_gpu_kernels.py
step search 600 $PYT tests/test_gpu_search.py tests/test_gpu_passes.py tests/test_gpu_rccl.py
step headline 400 $PYT tests/test_gpu_headline.py
for i in 1 2; do
  BRP_PHASES=1 WORK=/tmp/appb timeout -k 10 120 bash scripts/bench_single.sh > gpurun_out/r3_app$i.log 2>&1 \
    || { echo APP_FAIL; tail -20 /tmp/appb/app.log; exit 1; }
  cat gpurun_out/r3_app$i.log; grep "\[phase\]" /tmp/appb/app.log
done
if [ -z "${SKIP_PMC:-}" ]; then
  rm -rf gpurun_out/pmc3; mkdir -p gpurun_out/pmc3
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD \
    -d gpurun_out/pmc3 -o s1 --output-format csv -- python3 tools/stagebench.py 1 > gpurun_out/pmc3/s1.log 2>&1 || { echo PMC_FAIL; tail -20 gpurun_out/pmc3/s1.log; exit 1; }
  python3 scripts/pmc_summary.py gpurun_out/pmc3 > gpurun_out/pmc3_summary.txt
  grep -A9 "hs_pruned\|pass3_kernel<256, 8, 0>" gpurun_out/pmc3_summary.txt
fi
step bluestein 600 $PYT tests/test_gpu_bluestein.py
echo "failed steps:${FAILED:- none}"
