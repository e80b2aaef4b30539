#!/bin/bash
# One loop workgroup (32 x 64 shape, sps 8) with 8, 16, 24, 32 live streams:
# cycles per symbol against the number of active lanes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}; O=$R/gpurun_out; mkdir -p $O; cd $R
for i in 1 2; do
  for s in 8 16 20 24 28 32; do
    timeout -k 10 120 tools/bin/loop_probe $s 1048576 2 0 0 8.0 > $O/probe_lanes$s.txt 2>&1 || exit 1
    echo "S=$s $(grep 'rounds' $O/probe_lanes$s.txt | head -1 | grep -o 'cyc/sym.*')"
  done
done
