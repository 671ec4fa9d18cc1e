# Compute-only strong-scaling proxy on ONE GPU: for N = 1, 2, 4, 8 time every
# rank's actual template block of the N-rank bench (bench.py --shard-of N:R,
# no collectives) and take the slowest rank as the node step time. The
# all-gather of the 24 KB tables is not included; the driver's 8-GPU run is
# the measurement, this is a proxy.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for n in 1 2 4 8; do
  worst=0
  for r in $(seq 0 $((n - 1))); do
    timeout -k 10 200 python bench.py --steps ${STEPS:-3} --warmup 1 --shard-of $n:$r > gpurun_out/shard_${n}_$r.log 2>&1 || { echo "FAIL $n:$r"; tail -20 gpurun_out/shard_${n}_$r.log; exit 1; }
    ms=$(python3 -c "import json; print(json.loads(open('gpurun_out/shard_${n}_$r.log').read().strip().splitlines()[-1])['ms_per_step'])")
    echo "N=$n rank=$r ms/step=$ms"
    worst=$(python3 -c "print(max($worst, $ms))")
  done
  python3 -c "print(f'N=$n slowest rank {$worst} ms/step -> node estimate {6662*1e3/$worst:.0f} templates/s (compute-only, max over ranks)')"
done
