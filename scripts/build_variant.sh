#!/bin/bash
# Build an experiment variant of the native code for scripts/gpu_ab_so.sh:
#   scripts/build_variant.sh <name> "<extra compiler flags>"
# copies the tree (sources only) to /tmp/var_<name>, builds it there with
# BRP_EXTRA_CFLAGS, and puts the extension (and the app) into ab/<name>/.
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
name=$1; flags=${2:-}
W=/tmp/var_$name
rm -rf "$W"; mkdir -p "$W"
(cd "$ROOT" && tar --exclude=./ab --exclude=./gpurun_out --exclude=./build --exclude=./.git -cf - .) | tar -xf - -C "$W"
(cd "$W" && BRP_EXTRA_CFLAGS="$flags" python -c "from boinc_app_eah_brp_amd import _build; _build.build(force=True, verbose=False)")
mkdir -p "$ROOT/ab/$name/bin"
cp "$W"/boinc_app_eah_brp_amd/_brp*.so "$ROOT/ab/$name/"
cp "$W"/bin/einsteinbinary_mi355x "$ROOT/ab/$name/bin/"
echo "built ab/$name ($flags)"
