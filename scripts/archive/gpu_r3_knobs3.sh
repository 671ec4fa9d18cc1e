# Round 3: pass-2 persistence, batches in flight and pipelines re-checked at
# the current defaults (2 interleaved rounds each).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
EXPS="- BRP_PERSIST=2 BRP_PERSIST=6 BRP_PERSIST=0 BRP_INFLIGHT=3 BRP_STREAMS=4 - BRP_PERSIST=2 BRP_PERSIST=6 BRP_PERSIST=0 BRP_INFLIGHT=3 BRP_STREAMS=4" timeout -k 10 1000 bash scripts/gpu_ab_bench.sh || exit $?
