# PMC counters of the template pipeline kernels on the stage benchmark (batch 8)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/pmcf; mkdir -p gpurun_out/pmcf
set1="SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE"
set2="SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
set3="TA_TA_BUSY_sum TA_BUSY_avr TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
i=0
for set in "$set1" "$set2" "$set3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d gpurun_out/pmcf -o s$i --output-format csv -- python3 tools/stagebench.py 8 > gpurun_out/pmcf/s$i.log 2>&1 || { echo PMC_FAIL $i; tail -20 gpurun_out/pmcf/s$i.log; exit 1; }
done
python3 scripts/pmc_summary.py gpurun_out/pmcf > gpurun_out/pmcf/summary.txt
grep -A 26 "pass1_pruned3\|pass2r_kernel<128>\|pass3_kernel<256, 8, 0>\|harmonic_sum_kernel<float, false>" gpurun_out/pmcf/summary.txt
