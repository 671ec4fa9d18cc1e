# Harmonic-sum kernel A/B: kernel tests, stage benchmark and interleaved bench
# runs of the register-blocked (default) and gather kernels.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v -m gpu --timeout 120 --timeout-method thread -k harmonic \
  > gpurun_out/hs_tests.log 2>&1 || { echo TEST_FAIL; tail -60 gpurun_out/hs_tests.log; exit 1; }
tail -3 gpurun_out/hs_tests.log
for v in rb gather; do
  BRP_HS_KERNEL=$v timeout -k 10 120 python tools/stagebench.py 1 > gpurun_out/hs_stage_$v.json 2>&1 || { echo STAGE_FAIL $v; tail gpurun_out/hs_stage_$v.json; exit 1; }
  echo "$v $(tail -1 gpurun_out/hs_stage_$v.json)"
done
for rep in 1 2; do
  for v in rb gather; do
    BRP_HS_KERNEL=$v timeout -k 10 200 python bench.py --steps ${STEPS:-6} --warmup 2 > gpurun_out/hs_bench_${v}_$rep.json 2>gpurun_out/hs_bench_${v}_$rep.err || { echo BENCH_FAIL $v; tail gpurun_out/hs_bench_${v}_$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['recall_vs_golden'])" gpurun_out/hs_bench_${v}_$rep.json $v
  done
done
