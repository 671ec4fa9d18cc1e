# Round 3 re-entry: round-end rehearsal at HEAD (fresh build) + kernel stats of the bench.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
bash scripts/gpu_roundend.sh || exit 1
bash scripts/gpu_profile.sh
