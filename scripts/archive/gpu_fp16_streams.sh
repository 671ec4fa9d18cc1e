# Config 5 (fp16 spectrum): pipelines per GPU sweep (run via gpurun).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/fp16s
for s in 2 3 4 3; do
  timeout -k 10 200 python bench.py --steps 2 --warmup 1 --ps-fp16 --streams $s > gpurun_out/fp16s/s$s.log 2>&1 \
    || { echo BENCH_FAIL; tail -20 gpurun_out/fp16s/s$s.log; exit 1; }
  echo "streams=$s $(tail -1 gpurun_out/fp16s/s$s.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["recall_vs_golden"])')"
done
