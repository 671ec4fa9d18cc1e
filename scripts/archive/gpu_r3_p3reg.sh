# Round 3: pass 3 with its first radix-16 stage in registers from 8-byte row
# loads (ab/p3reg, -DBRP_P3_REG_STAGE1) vs 16-byte row loads into LDS (head).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
ROUNDS=3 timeout -k 10 600 bash scripts/gpu_ab_so.sh > gpurun_out/r3_p3reg_ab.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/r3_p3reg_ab.log; exit 1; }
grep round gpurun_out/r3_p3reg_ab.log
for v in head p3reg; do
  if [ $v = head ]; then d=$GRAFT_REPO_ROOT; else d=/tmp/ab_$v; fi
  (cd $d && timeout -k 10 120 python tools/stagebench.py 1) > gpurun_out/r3_p3reg_stage_$v.log 2>&1 || { echo STAGE_FAIL $v; tail gpurun_out/r3_p3reg_stage_$v.log; exit 1; }
  echo "stage $v $(tail -1 gpurun_out/r3_p3reg_stage_$v.log)"
done
