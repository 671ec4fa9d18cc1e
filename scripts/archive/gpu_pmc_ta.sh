# TA / TCP / GRBM counters per kernel on the stage benchmark
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/pmct; mkdir -p gpurun_out/pmct
i=0
for set in "GRBM_GUI_ACTIVE TA_BUSY_avr TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum" \
           "TCP_PENDING_STALL_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
           "SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_WAVE_CYCLES" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set -d gpurun_out/pmct -o s$i --output-format csv -- python3 tools/stagebench.py 4 > gpurun_out/pmct/s$i.log 2>&1 || { echo PMC_FAIL $i; tail -5 gpurun_out/pmct/s$i.log; }
done
python3 scripts/pmc_summary.py gpurun_out/pmct
