# Round 3: start-up tracing (scripts/gpu_r3_startup.sh), then speed-of-light
# ablations of the bench (ab/p3fft, p1fft, p1res, hsoff from
# scripts/build_variant.sh) against head, interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_r3_startup.sh || exit $?
ROUNDS=${ROUNDS:-2} timeout -k 10 900 bash scripts/gpu_ab_so.sh > gpurun_out/r3_sol_ab.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/r3_sol_ab.log; exit 1; }
grep round gpurun_out/r3_sol_ab.log
