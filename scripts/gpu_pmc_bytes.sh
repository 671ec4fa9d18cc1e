# HBM bytes (FETCH_SIZE / WRITE_SIZE, separate passes) and LDS/VALU counters
# per kernel on the stage benchmark at batch 1 (the default 1-template shape).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/pmcb; mkdir -p gpurun_out/pmcb
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d gpurun_out/pmcb -o s$i --output-format csv -- python3 tools/stagebench.py ${STAGE_BATCH:-1} > gpurun_out/pmcb/s$i.log 2>&1 || { echo PMC_FAIL $i; tail -20 gpurun_out/pmcb/s$i.log; exit 1; }
done
python3 scripts/pmc_summary.py gpurun_out/pmcb > gpurun_out/pmcb_summary.txt
cat gpurun_out/pmcb_summary.txt
tail -1 gpurun_out/pmcb/s1.log
