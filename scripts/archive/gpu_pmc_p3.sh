# Pass-3 counters: LDS-staged (BRP_P3R=0) vs register pass 3 (default), stage benchmark at batch 1.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/pmc3; mkdir -p gpurun_out/pmc3
i=0
for cfg in 0 16; do
for set in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" ; do
  i=$((i+1))
  BRP_P3R=$cfg timeout -s KILL 120 rocprofv3 --pmc $set -d gpurun_out/pmc3/c$cfg -o s$i --output-format csv -- python3 tools/stagebench.py 1 > gpurun_out/pmc3/s$i.log 2>&1 || { echo PMC_FAIL $i; tail -20 gpurun_out/pmc3/s$i.log; exit 1; }
done
python3 scripts/pmc_summary.py gpurun_out/pmc3/c$cfg > gpurun_out/pmc3_summary_$cfg.txt
grep -A20 "pass3" gpurun_out/pmc3_summary_$cfg.txt
done
