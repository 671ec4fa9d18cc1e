# Harmonic-sum variant experiments (tools/experiments/hs_variants, built on the
# CPU side): dump one benchmark-template spectrum, then time every variant and
# check it against the gather kernel, at low thresholds (many candidates) and
# at the search's chi^2 thresholds.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
geo=$(timeout -k 10 120 python tools/experiments/dump_ps.py /tmp/ps.f32 0 2>gpurun_out/dump_ps.err | tail -1) || { echo DUMP_FAIL; tail gpurun_out/dump_ps.err; exit 1; }
echo "geometry: $geo"
timeout -k 10 120 tools/experiments/hs_variants /tmp/ps.f32 $geo 200 9 12 16 22 33 | tee gpurun_out/hs_exp_low.json || exit 1
timeout -k 10 120 tools/experiments/hs_variants /tmp/ps.f32 $geo 200 18.139 21.241 26.269 34.648 48.958 | tee gpurun_out/hs_exp_chi2.json || exit 1
