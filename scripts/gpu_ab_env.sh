# A/B of runtime switches (and experiment builds) in one GPU call:
#   VARIANTS="name:VAR=v,VAR=v name2@build:VAR=v ..."
# name "head" = no extra environment; "@build" runs the ab/<build>/ extension
# from a copy of the tree. Each variant is a bench.py run, interleaved over
# $ROUNDS rounds.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
prep() {  # copy of the tree with ab/<build>'s extension
  local b=$1
  [ -d /tmp/ab_$b ] && return 0
  mkdir -p /tmp/ab_$b
  tar --exclude=./ab --exclude=./gpurun_out -cf - . | tar -xf - -C /tmp/ab_$b
  cp ab/$b/_brp*.so /tmp/ab_$b/boinc_app_eah_brp_amd/
}
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in ${VARIANTS:-head}; do
    nb=${v%%:*}; e=""
    [ "$nb" != "$v" ] && e=$(echo ${v#*:} | tr ',' ' ')
    n=${nb%%@*}; dir=$GRAFT_REPO_ROOT
    if [ "$n" != "$nb" ]; then prep ${nb#*@}; dir=/tmp/ab_${nb#*@}; fi
    (cd $dir && env $e timeout -k 10 200 python bench.py --steps ${STEPS:-2} --warmup 1 ${BENCH_ARGS:-}) > gpurun_out/abe_$n.log 2>&1 \
      || { echo "FAIL $n"; tail -20 gpurun_out/abe_$n.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[2]).read().strip().splitlines()[-1]); print(sys.argv[1], 'round', sys.argv[3], d['value'], d.get('recall_vs_golden'))" \
      "$n" gpurun_out/abe_$n.log $r
  done
done
