# Counter list of the box + SQ counters of the three harmonic-sum kernels on the stage benchmark.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmchs
timeout -s KILL 60 rocprofv3 --list-avail > gpurun_out/pmchs/avail.txt 2>&1 || echo LIST_FAIL
for v in gather quad rb; do
  BRP_HS_KERNEL=$v timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_WAIT_ANY -d gpurun_out/pmchs/$v -o s --output-format csv -- python3 tools/stagebench.py 1 > gpurun_out/pmchs/$v.log 2>&1 || { echo PMC_FAIL $v; tail -20 gpurun_out/pmchs/$v.log; exit 1; }
  echo "== $v"; python3 scripts/pmc_summary.py gpurun_out/pmchs/$v | grep -A9 harmonic_sum
done
