# one test in the tree's build and in ab/<variant> builds (copies of the tree under /tmp)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for d in ab/*/; do
  n=$(basename $d)
  rm -rf /tmp/ab_$n && mkdir -p /tmp/ab_$n
  tar --exclude=./ab --exclude=./gpurun_out -cf - . | tar -xf - -C /tmp/ab_$n
  cp $d/_brp*.so /tmp/ab_$n/boinc_app_eah_brp_amd/
  (cd /tmp/ab_$n && timeout -k 10 300 python -u -m pytest "$TEST" -x -q -m gpu --timeout 200 --timeout-method thread) > gpurun_out/one_$n.log 2>&1; echo "$n rc=$?"; grep -E "^E .*Assertion|passed|failed" gpurun_out/one_$n.log | head -3
done
timeout -k 10 300 python -u -m pytest "$TEST" -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/one_head.log 2>&1; echo "head rc=$?"; grep -E "^E .*Assertion|passed|failed" gpurun_out/one_head.log | head -3
