# PMC passes on the chirp-z path (one pipeline, bench.py --padding P) -> gpurun_out/pmcc_summary.txt
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/pmcc; mkdir -p gpurun_out/pmcc
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS" \
           "FETCH_SIZE" "WRITE_SIZE GRBM_GUI_ACTIVE" ; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $set -d gpurun_out/pmcc -o s$i --output-format csv -- python3 bench.py --steps 1 --warmup 0 --streams 1 --templates ${TEMPLATES:-60} --padding ${PADDING:-2.7} > gpurun_out/pmcc/s$i.log 2>&1 || { echo PMC_FAIL $i; tail -20 gpurun_out/pmcc/s$i.log; exit 1; }
done
python3 scripts/pmc_summary.py gpurun_out/pmcc > gpurun_out/pmcc_summary.txt
grep -A12 "pass1g_kernel<320, 6>\|pass3_mid\|pass2g_kernel<288, true" gpurun_out/pmcc_summary.txt
