# throughput vs device batch size and pipelines per GPU (MALL residency of the FFT buffers)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for cfg in ${CFGS:-1,2 1,4 2,2 2,3 2,4 4,2 4,3 8,2}; do
  set -- ${cfg/,/ }
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --batch $1 --streams $2 > gpurun_out/sweep_b$1_s$2.log 2>&1 || { echo FAIL $cfg; tail -20 gpurun_out/sweep_b$1_s$2.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/sweep_b$1_s$2.log').read().strip().splitlines()[-1]); print('batch',$1,'streams',$2,d['value'],d['phase_ms_per_step_rank0'])"
done
