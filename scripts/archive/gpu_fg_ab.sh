# Fine-grained result buffer (BRP_FG=both: the host reads the candidate list in
# place, no per-batch device->host copy) against the default (parameters in place).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2 3; do for f in in both; do
  BRP_FG=$f timeout -k 10 200 python bench.py --steps 8 --warmup 1 > gpurun_out/fg_$f.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/fg_$f.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/fg_$f.log').read().strip().splitlines()[-1]); print('fg=$f', d['value'], d['recall_vs_golden']['table'], d['table_identical_to_warmup'])"
done; done
