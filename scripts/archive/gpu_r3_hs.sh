# Round 3: conflict-free pruned harmonic-sum bound reads -- tests, A/B bench
# against ab/base (HEAD build), LDS counters of the stage benchmark.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_kernels.py -k "harmonic" tests/test_gpu_search.py -k "harmonic or oom" > gpurun_out/r3_tests.log 2>&1 \
  || { echo TEST_FAIL; tail -40 gpurun_out/r3_tests.log; exit 1; }
tail -2 gpurun_out/r3_tests.log
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_passes.py \
  > gpurun_out/r3_passes.log 2>&1 || { echo PASSES_FAIL; tail -40 gpurun_out/r3_passes.log; exit 1; }
tail -2 gpurun_out/r3_passes.log
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_gpu_headline.py \
  > gpurun_out/r3_headline.log 2>&1 || { echo HEADLINE_FAIL; tail -40 gpurun_out/r3_headline.log; exit 1; }
tail -2 gpurun_out/r3_headline.log
ROUNDS=3 bash scripts/gpu_ab_so.sh || exit 1
rm -rf gpurun_out/pmc3; mkdir -p gpurun_out/pmc3
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD \
  -d gpurun_out/pmc3 -o s1 --output-format csv -- python3 tools/stagebench.py 1 > gpurun_out/pmc3/s1.log 2>&1 || { echo PMC_FAIL; tail -20 gpurun_out/pmc3/s1.log; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/pmc3 > gpurun_out/pmc3_summary.txt
grep -A9 "hs_pruned\|pass3_kernel<256, 8, 0>" gpurun_out/pmc3_summary.txt
