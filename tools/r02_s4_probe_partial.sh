#!/bin/bash
# Is the last, partly filled loop workgroup slower per symbol?  S=256 (10 full
# workgroups of 24 streams + one of 16) against S=264 (11 full), sps 8.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}; O=$R/gpurun_out; mkdir -p $O; cd $R
for s in 256 264 256 264; do
  timeout -k 10 120 tools/bin/loop_probe $s 1048576 4 0 0 8.0 > $O/probe_p$s.txt 2>&1 || exit 1
  head -1 $O/probe_p$s.txt; grep -E "^ WG (10|1)[ :]" $O/probe_p$s.txt | cut -c1-40,150-; tail -1 $O/probe_p$s.txt
done
