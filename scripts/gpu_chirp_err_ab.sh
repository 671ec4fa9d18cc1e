set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for d in ab/*/; do
  n=$(basename $d)
  rm -rf /tmp/ab_$n && mkdir -p /tmp/ab_$n
  tar --exclude=./ab --exclude=./gpurun_out -cf - . | tar -xf - -C /tmp/ab_$n
  cp $d/_brp*.so /tmp/ab_$n/boinc_app_eah_brp_amd/
  echo "== $n"; (cd /tmp/ab_$n && timeout -k 10 400 python tools/chirp_err.py) 2>&1 | grep -E "max=|top bins|16ths" || exit 1
done
echo "== head"; timeout -k 10 400 python tools/chirp_err.py 2>&1 | grep -E "max=|top bins|16ths"
