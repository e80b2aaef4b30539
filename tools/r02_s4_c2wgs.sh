#!/bin/bash
# Loop time per call against the number of loop workgroups (sps 8, 24 x 128
# shape, 2^20 samples per stream): the per-stream chain is the same, so any
# growth is the chip's, not the kernel's.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}; O=$R/gpurun_out; mkdir -p $O; cd $R
run() { out=$(timeout -k 10 300 python3 bench.py --timed-only --config c2 --steps 6 --warmup 2 --loop-variant 4 --streams $1) || exit 1
  echo "streams $1 $(echo "$out" | grep -o '"loop": [0-9][0-9.]*' | head -1) $(echo "$out" | grep -o '"ms_per_step": [0-9.]*' | head -1)"; }
for i in 1 2; do
  for s in 24 96 256 512 1024 2048 4096; do run $s; done
done
