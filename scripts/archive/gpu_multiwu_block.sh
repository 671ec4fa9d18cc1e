# A/B of the multi-WU deal order (run via gpurun): BRP_MULTI_BLOCK=1 (old
# interleaved order) vs the default WU-major blocks, 8 WUs resident.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for blk in 1 64 1 64; do
  BRP_MULTI_BLOCK=$blk timeout -k 10 300 python bench.py --steps 1 --warmup 1 --wus ${WUS:-8} \
    > gpurun_out/mwu_blk$blk.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/mwu_blk$blk.log; exit 1; }
  echo "block=$blk $(tail -1 gpurun_out/mwu_blk$blk.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["unit"], d.get("recall_vs_golden"))')"
done
