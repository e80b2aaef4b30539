#!/bin/bash
# C4 shard (4096 streams, sps 8, 65 taps): loop shape 24 x 128 (auto today;
# 171 workgroups whose 147 KB of LDS leave no room for a FIR workgroup) vs
# 32 x 64 (128 workgroups, 104 KB).  A/B x2.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}; O=$R/gpurun_out; mkdir -p $O; cd $R
run() { out=$(timeout -k 10 300 python3 bench.py --timed-only --config c4 --streams $2 --steps 6 --warmup 2 --loop-variant $1) || exit 1
  echo "S=$2 v$1 $(echo "$out" | grep -o '"fir": [0-9][0-9.]*' | head -1) $(echo "$out" | grep -o '"loop": [0-9][0-9.]*' | head -1) $(echo "$out" | grep -o '"ms_per_step": [0-9.]*' | head -1) $(echo "$out" | grep -o '"value": [0-9.]*' | head -1)"; }
for i in 1 2; do
  for s in 4096 2048 1024; do
    for v in 4 2; do run $v $s; done
  done
done
