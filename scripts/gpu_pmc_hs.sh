# PMC counters of the harmonic-sum variants (staged / gather) on the stage benchmark
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/pmch; mkdir -p gpurun_out/pmch
set1="SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE"
set2="TCC_HIT_sum TCC_MISS_sum TA_TA_BUSY_sum TA_BUSY_avr GRBM_GUI_ACTIVE"
for v in staged gather; do
  envs=""; [ $v = gather ] && envs="BRP_HS_GATHER=1"
  i=0
  for set in "$set1" "$set2"; do
    i=$((i+1))
    env $envs timeout -s KILL 120 rocprofv3 --pmc $set -d gpurun_out/pmch/$v -o s$i --output-format csv -- python3 tools/stagebench.py 4 > gpurun_out/pmch/$v$i.log 2>&1 || { echo PMC_FAIL $v $i; tail -20 gpurun_out/pmch/$v$i.log; exit 1; }
  done
  echo "== $v"; python3 scripts/pmc_summary.py gpurun_out/pmch/$v | grep -A 14 harmonic
done
