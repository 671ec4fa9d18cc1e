# Harmonic-sum kernel A/B: exactness tests of every variant, stage benchmark,
# interleaved bench runs of quad / gather / rb.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v -m gpu --timeout 120 --timeout-method thread -k harmonic \
  > gpurun_out/hs_tests.log 2>&1 || { echo TEST_FAIL; tail -60 gpurun_out/hs_tests.log; exit 1; }
tail -2 gpurun_out/hs_tests.log
run() {
  local name=$1; shift
  env "$@" timeout -k 10 120 python tools/stagebench.py 1 > gpurun_out/ab_stage_$name.json 2>&1 || { echo STAGE_FAIL $name; tail gpurun_out/ab_stage_$name.json; return 1; }
  echo "$name $(tail -1 gpurun_out/ab_stage_$name.json)"
}
bench() {
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps ${STEPS:-6} --warmup 2 > gpurun_out/ab_bench_$name.json 2>gpurun_out/ab_bench_$name.err || { echo BENCH_FAIL $name; tail gpurun_out/ab_bench_$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['recall_vs_golden']['table'])" gpurun_out/ab_bench_$name.json $name
}
run quad BRP_HS_KERNEL=quad && run gather BRP_HS_KERNEL=gather && run rb BRP_HS_KERNEL=rb || exit 1
for rep in 1 2; do
  bench quad_$rep BRP_HS_KERNEL=quad && bench gather_$rep BRP_HS_KERNEL=gather || exit 1
done
