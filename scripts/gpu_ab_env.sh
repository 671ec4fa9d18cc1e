# A/B of runtime switches in one GPU call: VARIANTS="name:VAR=v,VAR=v name2:..." (name "head" = no
# extra environment), each a bench.py run, interleaved over $ROUNDS rounds.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in ${VARIANTS:-head}; do
    n=${v%%:*}; e=""
    [ "$n" != "$v" ] && e=$(echo ${v#*:} | tr ',' ' ')
    env $e timeout -k 10 200 python bench.py --steps ${STEPS:-2} --warmup 1 ${BENCH_ARGS:-} > gpurun_out/abe_$n.log 2>&1 \
      || { echo "FAIL $n"; tail -20 gpurun_out/abe_$n.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[2]).read().strip().splitlines()[-1]); print(sys.argv[1], 'round', sys.argv[3], d['value'], d.get('recall_vs_golden'))" \
      "$n" gpurun_out/abe_$n.log $r
  done
done
