# Kernel stats of the bench for head, each ab/<name> build and each ENV variant (KVARIANTS="name:VAR=v ...").
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {  # run <name> <dir> <env...>
  local n=$1 dir=$2; shift 2
  rm -rf gpurun_out/ks_$n; mkdir -p gpurun_out/ks_$n
  (cd $dir && env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/ks_$n -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1) > gpurun_out/ks_$n.log 2>&1 || { echo "FAIL $n"; tail -20 gpurun_out/ks_$n.log; exit 1; }
  echo "== $n: $(tail -1 gpurun_out/ks_$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d.get("recall_vs_golden"))')"
  python3 scripts/kstats.py $(find gpurun_out/ks_$n -name '*kernel_stats.csv' | head -1) | head -6
}
run head $GRAFT_REPO_ROOT BRP_NOP=1
for d in ab/*/; do
  [ -d "$d" ] || continue
  n=$(basename $d)
  rm -rf /tmp/ab_$n && mkdir -p /tmp/ab_$n
  tar --exclude=./ab --exclude=./gpurun_out -cf - . | tar -xf - -C /tmp/ab_$n
  cp $d/_brp*.so /tmp/ab_$n/boinc_app_eah_brp_amd/
  run $n /tmp/ab_$n BRP_NOP=1
done
for v in ${KVARIANTS:-}; do
  n=${v%%:*}; e=$(echo ${v#*:} | tr ',' ' ')
  run $n $GRAFT_REPO_ROOT $e
done
