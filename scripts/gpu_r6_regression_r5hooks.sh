#!/bin/bash
# Round 6 regression check: the checked-build test of the benchmark batch run
# against a checked build whose bound_cells copies into the caller's pageable
# vector again (the round-5 form, ab/r5hooks, built by patching hip_engine.cpp
# in a copy of the tree). Expected: test_checked_bench_batch_clean FAILS with
# the checked build's "pageable memory" report -- i.e. the test catches the
# round-5 engine deterministically.
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
W=/tmp/r5hooks
rm -rf "$W" && mkdir -p "$W"
(cd "$ROOT" && tar --exclude=./ab --exclude=./gpurun_out -cf - .) | tar -xf - -C "$W"
cp "$ROOT"/ab/r5hooks/_brp_checked*.so "$W/boinc_app_eah_brp_amd/"
cd "$W"
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_checked.py::test_checked_bench_batch_clean -x -v --timeout 150 \
  --timeout-method thread > "$ROOT/gpurun_out/r5hooks_test.log" 2>&1
rc=$?
echo "round-5 hooks, checked test rc=$rc (1 = the test failed, as expected)"
grep -o "checked: a host copy[^\"']*" "$ROOT/gpurun_out/r5hooks_test.log" | head -3
[ $rc -eq 0 ] || [ $rc -eq 1 ]
