#!/bin/bash
# Occupancy and latency counters of the harmonic-sum kernels (round-6 verdict
# item 5): SQ_WAVE_CYCLES, SQ_WAIT_INST_ANY, SQ_INSTS_VMEM_RD and friends in one
# pass (8 SQ counters), bench geometry, one pipeline, 60 templates
# -> gpurun_out/pmchs6_summary.txt
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
rm -rf gpurun_out/pmchs6; mkdir -p gpurun_out/pmchs6
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU \
  -d gpurun_out/pmchs6 -o hs --output-format csv -- python3 bench.py --steps 1 --warmup 0 --streams 1 --templates 60 > gpurun_out/pmchs6/run.log 2>&1 || { echo PMC_FAIL; tail -20 gpurun_out/pmchs6/run.log; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/pmchs6 > gpurun_out/pmchs6_summary.txt
grep -A10 "hs_pruned\|hs_cells\|pass3_kernel<256, 8, 0" gpurun_out/pmchs6_summary.txt
