# Round 3: HIP start-up pieces (tools/experiments/startup/startup_bench.hip),
# sequential vs one thread per stream, fresh process each.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for m in seq par seq par seq par; do
  timeout -k 10 60 build/exp/startup_bench $m 3 || { echo FAIL $m; exit 1; }
done
for m in seq par; do
  t0=$(date +%s%N); timeout -k 10 60 build/exp/startup_bench $m 3 > /dev/null; t1=$(date +%s%N)
  echo "$m process wall incl. exit: $(( (t1 - t0) / 1000000 )) ms"
done
