# Harmonic-sum kernel A/B (stage benchmark + interleaved bench): register-blocked
# with free / 4-wave occupancy, and the per-i gather kernel.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python tools/stagebench.py 1 > gpurun_out/ab_stage_$name.json 2>&1 || { echo STAGE_FAIL $name; tail gpurun_out/ab_stage_$name.json; return 1; }
  echo "$name $(tail -1 gpurun_out/ab_stage_$name.json)"
}
bench() {
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps ${STEPS:-6} --warmup 2 > gpurun_out/ab_bench_$name.json 2>gpurun_out/ab_bench_$name.err || { echo BENCH_FAIL $name; tail gpurun_out/ab_bench_$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['recall_vs_golden']['table'])" gpurun_out/ab_bench_$name.json $name
}
run rb BRP_HS_KERNEL=rb && run rb4 BRP_HS_KERNEL=rb BRP_HS_RB_OCC=4 && run gather BRP_HS_KERNEL=gather || exit 1
for rep in 1 2; do
  bench rb4_$rep BRP_HS_KERNEL=rb BRP_HS_RB_OCC=4 && bench gather_$rep BRP_HS_KERNEL=gather && bench rb_$rep BRP_HS_KERNEL=rb || exit 1
done
