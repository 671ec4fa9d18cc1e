# Round 3: HS / pass ablations (ab/*) against head, then start-up tracing
# with a normal exit (so rocprofv3 writes its trace).
set -o pipefail
cd $GRAFT_REPO_ROOT
ROUNDS=${ROUNDS:-2} timeout -k 10 900 bash scripts/gpu_ab_so.sh > gpurun_out/r3_sol_ab2.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/r3_sol_ab2.log; exit 1; }
grep round gpurun_out/r3_sol_ab2.log
MEMBENCH_SIZES=1 bash scripts/gpu_r3_startup.sh
