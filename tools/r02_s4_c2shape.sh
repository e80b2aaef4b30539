#!/bin/bash
# C2 loop shapes: 4 = 24 x 128 (11 workgroups, the default at sps 8),
# 3 = 16 x 128 (16 workgroups), 1 = 16 x 64 (16), 2 = 32 x 64 (8).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}; O=$R/gpurun_out; mkdir -p $O; cd $R
run() { out=$(timeout -k 10 300 python3 bench.py --timed-only --config c2 --steps 10 --warmup 2 --loop-variant $1) || exit 1
  echo "c2 v$1 $(echo "$out" | grep -o '"loop": [0-9][0-9.]*' | head -1) $(echo "$out" | grep -o '"ms_per_step": [0-9.]*' | head -1) $(echo "$out" | grep -o '"value": [0-9.]*' | head -1)"; }
for i in 1 2 3; do
  for v in 4 3 1 2; do run $v; done
done
