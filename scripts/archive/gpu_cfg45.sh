# Config 4 at 64 resident WUs, and per-kernel stats of config 5 (fp16 power
# spectrum) vs the fp32 default on the same 600-template slice (run via gpurun).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cfg45
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/cfg45/fp32 -o run -- \
  python3 bench.py --steps 1 --warmup 0 --templates 600 > gpurun_out/cfg45/fp32.log 2>&1 || { echo FP32_FAIL; tail -20 gpurun_out/cfg45/fp32.log; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/cfg45/fp16 -o run -- \
  python3 bench.py --steps 1 --warmup 0 --templates 600 --ps-fp16 > gpurun_out/cfg45/fp16.log 2>&1 || { echo FP16_FAIL; tail -20 gpurun_out/cfg45/fp16.log; exit 1; }
timeout -k 10 240 python bench.py --steps 2 --warmup 1 --ps-fp16 > gpurun_out/cfg45/fp16_bench.log 2>&1 || { echo FP16B_FAIL; tail -20 gpurun_out/cfg45/fp16_bench.log; exit 1; }
tail -1 gpurun_out/cfg45/fp16_bench.log
timeout -k 10 600 python -u bench.py --steps 1 --warmup 1 --wus 64 > gpurun_out/cfg45/wus64.log 2>&1 || { echo WUS64_FAIL; tail -20 gpurun_out/cfg45/wus64.log; exit 1; }
tail -1 gpurun_out/cfg45/wus64.log
