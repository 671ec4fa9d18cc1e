set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for P in 2.7 2.9 1.1; do
  ROUNDS=1 STEPS=1 BENCH_ARGS="--padding $P" bash scripts/gpu_ab_so.sh || exit 1
done
