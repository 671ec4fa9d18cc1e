# Round 3: candidate list read in place (BRP_FG=both) vs the 8 KB copy per
# batch: search tests with it, 5 interleaved rounds.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 env BRP_FG=both python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_search.py tests/test_gpu_headline.py > gpurun_out/r3_fg_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r3_fg_tests.log; [ $rc -eq 0 ] || exit $rc
EXPS="- BRP_FG=both - BRP_FG=both - BRP_FG=both - BRP_FG=both - BRP_FG=both" timeout -k 10 900 bash scripts/gpu_ab_bench.sh || exit $?
