# Per-rank step time at the shard sizes of the 1/2/4/8-GPU strong-scaling bench
# (6662 / N templates on one GPU): the compute-only upper bound of each N.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for n in 1 2 4 8; do
  t=$(( (6662 + n - 1) / n ))
  timeout -k 10 200 python bench.py --steps 5 --warmup 2 --templates $t > gpurun_out/shard_$n.log 2>&1 || { echo "FAIL $n"; tail -20 gpurun_out/shard_$n.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/shard_$n.log').read().strip().splitlines()[-1]); n=int(sys.argv[1]); print(f'N={n} shard={d[\"config\"][\"global_batch\"]} ms/step={d[\"ms_per_step\"]} per-GPU t/s={d[\"value\"]:.0f} node estimate t/s={6662*1e3/d[\"ms_per_step\"]:.0f} phases={d[\"phase_ms_per_step_rank0\"]}')" $n
done
