# A/B full-bench comparison: one bench run per env setting in $EXPS ("-" = defaults)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for e in ${EXPS:--}; do
  if [ "$e" = "-" ]; then envs=""; else envs="${e//,/ }"; fi
  env $envs timeout -k 10 200 python bench.py --steps 2 --warmup 1 $BENCH_ARGS > gpurun_out/ab.log 2>&1 || { echo "FAIL $e"; tail -20 gpurun_out/ab.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d.get('recall_vs_golden'))" "$e"
done
