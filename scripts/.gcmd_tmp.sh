export TMPDIR=/tmp
timeout -k 10 60 ./build/probe/slab_scatter; timeout -k 10 60 ./build/probe/slab_scatter
bash scripts/gpu_roundend.sh
