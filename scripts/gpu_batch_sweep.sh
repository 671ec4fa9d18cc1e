set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for b in 1 2 4 8; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 2 --warmup 1 --batch $b > gpurun_out/bench_b$b.log 2>&1 || { echo FAIL $b; tail -20 gpurun_out/bench_b$b.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_b$b.log').read().strip().splitlines()[-1]); print('batch',$b,d['value'],d['ms_per_step'],d['gpu_ms_rank0'])"
done
