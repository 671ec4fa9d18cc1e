# Round 3: Infinity-Cache-resident vs HBM copy bandwidth (tools/membench.hip at
# 1/2/4/16 templates of buffer) and where the application's start-up time goes
# (exec + dynamic loading without the GPU, loader statistics, a HIP API trace
# of the reference bench protocol).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for b in ${MEMBENCH_SIZES:-1 2 4 16}; do
  timeout -k 10 60 build/exp/membench $b > gpurun_out/membench_$b.log 2>&1 || { echo MEMBENCH_FAIL $b; cat gpurun_out/membench_$b.log; exit 1; }
  echo "== membench $b"; head -4 gpurun_out/membench_$b.log
done
APP=bin/einsteinbinary_mi355x
for i in 1 2 3; do
  t0=$(date +%s%N); $APP --version > /dev/null 2>&1; t1=$(date +%s%N)
  echo "version run (exec, dynamic loading, static init, exit; no GPU use): $(( (t1 - t0) / 1000 )) us"
done
LD_DEBUG=statistics $APP --version > /dev/null 2> gpurun_out/ld_stats.log; grep -E "total startup|relocation|load" gpurun_out/ld_stats.log | head -12
ldd $APP > gpurun_out/ldd.txt; wc -l < gpurun_out/ldd.txt
D=data/testwu
W=/tmp/apptrace; mkdir -p $W
for i in 1 2; do
  BRP_PHASES=1 WORK=/tmp/appb timeout -k 10 120 bash scripts/bench_single.sh > gpurun_out/startup_app$i.log 2>&1 || { echo APP_FAIL; tail -20 /tmp/appb/app.log; exit 1; }
  cat gpurun_out/startup_app$i.log; grep "\[phase\]" /tmp/appb/app.log
done
rm -rf gpurun_out/apitrace
(cd $W && BRP_PHASES=1 BRP_FAST_EXIT=0 timeout -k 10 180 rocprofv3 --hip-trace --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/apitrace -o app --output-format csv -- \
  $GRAFT_REPO_ROOT/$APP -i $GRAFT_REPO_ROOT/$D/p2030.20151015.G187.41-00.88.N.b2s0g0.00000_1099.bin4 -t $GRAFT_REPO_ROOT/$D/stochastic_full.bank \
  -l $GRAFT_REPO_ROOT/$D/p2030.20151015.G187.41-00.88.N.b2s0g0.00000.zap -o results.cand -c checkpoint.cpt -A 0.08 -P 3.0 -f 400.0 -W \
  > $GRAFT_REPO_ROOT/gpurun_out/apitrace_app.log 2>&1) || { echo TRACE_FAIL; tail -20 gpurun_out/apitrace_app.log; exit 1; }
grep "\[phase\]" gpurun_out/apitrace_app.log
python3 scripts/api_timeline.py gpurun_out/apitrace 0.5 > gpurun_out/api_timeline.txt
head -80 gpurun_out/api_timeline.txt
