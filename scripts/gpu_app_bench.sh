# The BOINC application on the reference benchmark protocol (scripts/bench_single.sh),
# two batches in flight (default) vs one, plus a result-file check against the golden file.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for e in BRP_INFLIGHT=2 BRP_INFLIGHT=1 BRP_INFLIGHT=2; do
  env $e WORK=/tmp/appb timeout -k 10 200 bash scripts/bench_single.sh > gpurun_out/app_bench.log 2>&1 || { echo "APP FAIL $e"; tail -20 gpurun_out/app_bench.log; tail -20 /tmp/appb/app.log; exit 1; }
  echo "$e $(grep -E 'bench_single|Throughput' gpurun_out/app_bench.log | tr '\n' ' ')"
done
ls data/golden/ | head -5
