# GPU tests at HEAD, then an interleaved A/B of the round-3 session-2 switches.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
rc=$?
tail -2 gpurun_out/ab_tests.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/ab_tests.log | head -30; exit $rc; fi
VARIANTS="${VARIANTS:-head old:BRP_SERIAL=1,BRP_P3CELLS=0 s1:BRP_SERIAL=1 nop3:BRP_P3CELLS=0 s8:BRP_SERIAL=8}" ROUNDS=${ROUNDS:-3} bash scripts/gpu_ab_env.sh
