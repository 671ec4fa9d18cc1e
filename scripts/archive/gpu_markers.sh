# roctx ranges (BRP_ROCTX=1) + kernel trace of one bench step -> gpurun_out/markers
set -o pipefail
export TMPDIR=/tmp
export BRP_ROCTX=1
cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/markers; mkdir -p gpurun_out/markers
timeout -k 10 600 rocprofv3 --kernel-trace --marker-trace --stats -d gpurun_out/markers -o run --output-format csv -- python3 bench.py --gpus 1 --steps 1 --warmup 1 ${BENCH_ARGS:-} > gpurun_out/markers.log 2>&1 || { echo MARK_FAIL; tail -30 gpurun_out/markers.log; exit 1; }
tail -1 gpurun_out/markers.log
f=$(find gpurun_out/markers -name '*marker_api_trace.csv' | head -1)
head -2 "$f"
python3 scripts/marker_stats.py "$f"
# keep the merged-back output small: drop the big per-kernel trace
find gpurun_out/markers -name '*kernel_trace.csv' -delete
