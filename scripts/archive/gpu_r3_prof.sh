# Round 3 profiling: isolated per-stage times for each build (ab/* and head),
# kernel trace + stats of the head bench, the MFMA row-FFT experiment.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
names="head"
for d in ab/*/; do
  [ -d "$d" ] || continue
  n=$(basename $d)
  rm -rf /tmp/ab_$n && mkdir -p /tmp/ab_$n
  tar --exclude=./ab --exclude=./gpurun_out -cf - . | tar -xf - -C /tmp/ab_$n
  cp $d/_brp*.so /tmp/ab_$n/boinc_app_eah_brp_amd/
  names="$names $n"
done
for r in 1 2; do
  for n in $names; do
    if [ "$n" = head ]; then dir=$GRAFT_REPO_ROOT; else dir=/tmp/ab_$n; fi
    (cd $dir && timeout -k 10 120 python tools/stagebench.py 1) > gpurun_out/stage_$n.log 2>&1 || { echo "STAGE FAIL $n"; tail -20 gpurun_out/stage_$n.log; exit 1; }
    echo "stage $n $(tail -1 gpurun_out/stage_$n.log)"
  done
done
if [ -x build/exp/mfma_rowfft ]; then
  timeout -k 10 120 build/exp/mfma_rowfft > gpurun_out/mfma_rowfft.log 2>&1 || { echo MFMA_FAIL; tail -20 gpurun_out/mfma_rowfft.log; exit 1; }
  cat gpurun_out/mfma_rowfft.log
fi
bash scripts/gpu_profile.sh
