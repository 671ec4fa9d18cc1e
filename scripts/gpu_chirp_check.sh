# chirp-z path: GPU tests (SKIP_TESTS=1: none), then the bench rate per padding
# for each variant (VARIANTS="name:VAR=v,VAR=v ..."; "head" = defaults), then
# isolated kernel times (SKIP_PROF=1: none)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu_bluestein.py tests/test_gpu_radix7.py -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/chirp_tests.log 2>&1 || { echo TEST_FAIL; tail -60 gpurun_out/chirp_tests.log; exit 1; }
  tail -1 gpurun_out/chirp_tests.log
fi
for P in ${PADDINGS:-2.7 2.9 1.1}; do
  for v in ${VARIANTS:-head rev0:BRP_BS_REV=0}; do
    n=${v%%:*}; e=""
    [ "$n" != "$v" ] && e=$(echo ${v#*:} | tr ',' ' ')
    env $e timeout -k 10 200 python bench.py --steps 1 --warmup 1 --padding $P > gpurun_out/chirp_b_${P}_$n.log 2>&1 || { echo BFAIL $P $n; tail -20 gpurun_out/chirp_b_${P}_$n.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('P', sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'])" gpurun_out/chirp_b_${P}_$n.log $P $n
  done
done
[ -n "${SKIP_PROF:-}" ] || PADDINGS="2.7 2.9" bash scripts/gpu_prof_iso.sh
