# Serial launch groups: GPU tests at the default, then BRP_SERIAL A/B (interleaved).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ser_tests.log 2>&1
rc=$?
tail -3 gpurun_out/ser_tests.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error" gpurun_out/ser_tests.log | head -20; [ $rc -ne 1 ] && exit $rc; fi
VARIANTS="${VARIANTS:-s1:BRP_SERIAL=1 s2:BRP_SERIAL=2 head s8:BRP_SERIAL=8}" ROUNDS=${ROUNDS:-3} bash scripts/gpu_ab_env.sh
