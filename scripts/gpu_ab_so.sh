# A/B of native builds in one GPU call: every directory ab/<name>/ holding a
# built _brp*.so (and optionally bin/) is benchmarked against the tree's own
# build ("head"), interleaved over $ROUNDS rounds (cdna_hip_programming.md
# rule 24: deltas only from interleaved rounds in one process set).
# Variants run from copies of the tree under /tmp so that the package import
# picks up their .so.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
names="head"
for d in ab/*/; do
  [ -d "$d" ] || continue
  n=$(basename $d)
  rm -rf /tmp/ab_$n && mkdir -p /tmp/ab_$n
  tar --exclude=./ab --exclude=./gpurun_out -cf - . | tar -xf - -C /tmp/ab_$n
  cp $d/_brp*.so /tmp/ab_$n/boinc_app_eah_brp_amd/
  [ -d $d/bin ] && cp $d/bin/* /tmp/ab_$n/bin/
  names="$names $n"
done
for r in $(seq 1 ${ROUNDS:-2}); do
  for n in $names; do
    if [ "$n" = head ]; then dir=$GRAFT_REPO_ROOT; else dir=/tmp/ab_$n; fi
    (cd $dir && env ${ENVS:-} timeout -k 10 200 python bench.py --steps ${STEPS:-2} --warmup 1 $BENCH_ARGS) \
      > gpurun_out/ab_$n.log 2>&1 || { echo "FAIL $n"; tail -20 gpurun_out/ab_$n.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[2]).read().strip().splitlines()[-1]); print(sys.argv[1], 'round', sys.argv[3], d['value'], d.get('recall_vs_golden'))" \
      "$n" gpurun_out/ab_$n.log $r
  done
done
