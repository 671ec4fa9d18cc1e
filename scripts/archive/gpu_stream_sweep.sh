set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for cfg in "4 1" "4 2" "8 1" "8 2" "4 3"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --gpus 1 --steps 2 --warmup 1 --batch $1 --streams $2 > gpurun_out/bench_b$1_s$2.log 2>&1 || { echo FAIL $cfg; tail -20 gpurun_out/bench_b$1_s$2.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_b$1_s$2.log').read().strip().splitlines()[-1]); print('batch',$1,'streams',$2,d['value'],d['ms_per_step'],d['gpu_ms_rank0'])"
done
