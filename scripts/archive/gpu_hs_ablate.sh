# Harmonic-sum stage ablation (stage benchmark, batch 1): chi^2 thresholds x
# 1 (normal), x 0.8 (more flagged blocks), x 1000 (no exact work), per cell width
# and for the full gather kernel.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for cfg in "BRP_HS_CELL=8" "BRP_HS_CELL=4" "BRP_HS_FULL=1"; do
  for sc in 1 0.8 1000; do
    env $cfg BRP_STAGE_THR_SCALE=$sc timeout -k 10 120 python tools/stagebench.py 1 > gpurun_out/stage_abl.log 2>&1 || { echo "FAIL $cfg $sc"; tail -20 gpurun_out/stage_abl.log; exit 1; }
    echo "$cfg scale=$sc $(tail -1 gpurun_out/stage_abl.log)"
  done
done
