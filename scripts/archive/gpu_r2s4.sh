# Round 2, fourth session: round-end rehearsal, then kernel stats of the bench
# (pruned harmonic sum default) -> gpurun_out/prof
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
bash scripts/gpu_roundend.sh || exit 1
bash scripts/gpu_profile.sh || exit 1
