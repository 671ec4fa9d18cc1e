# Round 3: what the process exit of a HIP program costs (kernel-side GPU
# teardown after _exit) with nothing freed, buffers freed, buffers and
# streams destroyed; 3 streams x 80 MB like the application's pipelines.
set -o pipefail
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
  for td in none free all; do
    for mb in 80 4; do
      t0=$(date +%s%N)
      out=$(timeout -k 10 60 build/exp/startup_bench seq 3 $td $mb) || { echo FAIL; exit 1; }
      t1=$(date +%s%N)
      python3 -c "
import json,sys
d=json.loads(sys.argv[1]); t0=int(sys.argv[2])/1e6; t1=int(sys.argv[3])/1e6
print(f\"teardown={d['teardown']:5s} MB/stream={sys.argv[4]:>3s} in-process teardown {d['teardown_ms']:6.2f} ms, exit {t1-d['epoch_ms_before_exit']:6.1f} ms, process {t1-t0:6.1f} ms (init {d['init_ms']:.0f}, pipes {d['pipes_ms']:.0f})\")
" "$out" $t0 $t1 $mb
    done
  done
done
