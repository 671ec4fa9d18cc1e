# Round 3: L2 hit rate and memory-side requests per kernel at the default
# config (stage benchmark, one template per batch), one counter pass.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -rf gpurun_out/pmcl2; mkdir -p gpurun_out/pmcl2
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  -d gpurun_out/pmcl2 -o l2 --output-format csv -- python3 tools/stagebench.py 1 > gpurun_out/pmcl2/run.log 2>&1 || { echo PMC_FAIL; tail -20 gpurun_out/pmcl2/run.log; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/pmcl2 > gpurun_out/pmcl2_summary.txt
cat gpurun_out/pmcl2_summary.txt | head -80
