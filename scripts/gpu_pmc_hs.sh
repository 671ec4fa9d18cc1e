# L2 requests / hits of the harmonic-sum kernels at HEAD (bench geometry, one
# pipeline, 60 templates), one counter pass -> gpurun_out/pmchs_summary.txt
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/pmchs; mkdir -p gpurun_out/pmchs
timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE \
  -d gpurun_out/pmchs -o hs --output-format csv -- python3 bench.py --steps 1 --warmup 0 --streams 1 --templates 60 > gpurun_out/pmchs/run.log 2>&1 || { echo PMC_FAIL; tail -20 gpurun_out/pmchs/run.log; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/pmchs > gpurun_out/pmchs_summary.txt
grep -A12 "hs_pruned\|hs_cells" gpurun_out/pmchs_summary.txt
