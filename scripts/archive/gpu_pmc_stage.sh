# PMC counters per kernel on the stage benchmark (counters only, no trace domains)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmcs
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY" \
           "FETCH_SIZE WRITE_SIZE SQ_INSTS_SMEM SQ_WAIT_INST_LDS" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set -d gpurun_out/pmcs -o s$i --output-format csv -- python3 tools/stagebench.py 4 > gpurun_out/pmcs/s$i.log 2>&1 || { echo PMC_FAIL $i; tail -20 gpurun_out/pmcs/s$i.log; exit 1; }
done
python3 scripts/pmc_summary.py gpurun_out/pmcs
