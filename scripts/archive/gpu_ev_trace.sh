# Kernel traces of the bench under each BRP_EV mode (per-stream gaps), then an interleaved A/B.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for m in 0 1 2; do
  rm -rf gpurun_out/evt$m; mkdir -p gpurun_out/evt$m
  BRP_EV=$m timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/evt$m -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/evt$m.log 2>&1 || { echo TRACE_FAIL $m; tail -20 gpurun_out/evt$m.log; exit 1; }
  echo "== BRP_EV=$m $(tail -1 gpurun_out/evt$m.log | cut -c1-200)"
  python3 scripts/stream_gaps.py $(find gpurun_out/evt$m -name '*kernel_trace.csv' | head -1) | grep -E "queue|pass1_pruned|span"
done
VARIANTS="head ev1:BRP_EV=1 ev2:BRP_EV=2" ROUNDS=3 bash scripts/gpu_ab_env.sh
