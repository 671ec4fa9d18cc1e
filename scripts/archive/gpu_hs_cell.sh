# Pruned harmonic sum, level-4 bound over its own 16 indices: 4-bin (default)
# vs 8-bin bound cells, and the full gather kernel; tests, bench A/B in one
# call, kernel stats of the default.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -v -m gpu --timeout 120 --timeout-method thread \
  -k "harmonic" > gpurun_out/hsc_tests.log 2>&1 || { echo TEST_FAIL; tail -60 gpurun_out/hsc_tests.log; exit 1; }
tail -2 gpurun_out/hsc_tests.log
for r in 1 2; do
  for e in BRP_HS_CELL=8 BRP_HS_CELL=4; do
    env $e timeout -k 10 200 python bench.py --steps 4 --warmup 1 > gpurun_out/bench_hsc.log 2>&1 || { echo "BENCH FAIL $e"; tail -20 gpurun_out/bench_hsc.log; exit 1; }
    echo "bench $e $(python -c "import json,sys; d=json.loads(open('gpurun_out/bench_hsc.log').read().strip().splitlines()[-1]); print(d['value'], d['recall_vs_golden'], d['table_identical_to_warmup'])")"
  done
done
bash scripts/gpu_profile.sh
BENCH_ARGS="" bash -c 'BRP_HS_CELL=8 bash scripts/gpu_profile.sh' | grep -E "hs_|pass3_kernel<256, 8, 0>"
