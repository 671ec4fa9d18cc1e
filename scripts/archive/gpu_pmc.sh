set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS -d gpurun_out/pmc -o p1 --output-format csv -- python3 bench.py --gpus 1 --steps 1 --warmup 0 --templates 40 > gpurun_out/pmc1.log 2>&1 || { echo PMC1_FAIL; tail -20 gpurun_out/pmc1.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d gpurun_out/pmc -o p2 --output-format csv -- python3 bench.py --gpus 1 --steps 1 --warmup 0 --templates 40 > gpurun_out/pmc2.log 2>&1 || { echo PMC2_FAIL; tail -20 gpurun_out/pmc2.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc -o p3 --output-format csv -- python3 bench.py --gpus 1 --steps 1 --warmup 0 --templates 40 > gpurun_out/pmc3.log 2>&1 || { echo PMC3_FAIL; tail -20 gpurun_out/pmc3.log; exit 1; }
ls gpurun_out/pmc
