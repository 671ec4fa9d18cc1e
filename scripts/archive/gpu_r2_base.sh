# Round-2 baseline on a fresh box: round-end rehearsal (tests, smoke, bench),
# kernel stats of the default bench, and HBM bytes / LDS conflict counters per
# kernel on the stage benchmark at batch 1 (the 1-template x 3-pipeline default).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash scripts/gpu_roundend.sh || exit 1
bash scripts/gpu_profile.sh > gpurun_out/prof_summary.txt 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/prof_summary.txt; exit 1; }
tail -25 gpurun_out/prof_summary.txt
rm -rf gpurun_out/pmcb; mkdir -p gpurun_out/pmcb
i=0
for set in "FETCH_SIZE WRITE_SIZE" \
           "SQ_WAVES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD" ; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set -d gpurun_out/pmcb -o s$i --output-format csv -- python3 tools/stagebench.py 1 > gpurun_out/pmcb/s$i.log 2>&1 || { echo PMC_FAIL $i; tail -20 gpurun_out/pmcb/s$i.log; exit 1; }
done
python3 scripts/pmc_summary.py gpurun_out/pmcb > gpurun_out/pmcb_summary.txt
cat gpurun_out/pmcb_summary.txt
