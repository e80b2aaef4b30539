#!/bin/bash
# Stamped loop kernel (tools/loop_probe.hip) at several batch sizes, sps 8,
# 24 x 128 shape: cycles per symbol and the effective clock (s_memtime
# cycles over the event time), and where the workgroups ran.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}; O=$R/gpurun_out; mkdir -p $O; cd $R
for s in 24 96 256 1024 4096; do
  timeout -k 10 120 tools/bin/loop_probe $s 1048576 4 0 0 8.0 > $O/probe_s$s.txt 2>&1 || exit 1
  head -1 $O/probe_s$s.txt
done
timeout -k 10 120 tools/bin/loop_probe 256 1048576 4 200 0 8.0 > $O/probe_s256_burn.txt 2>&1 || exit 1
head -1 $O/probe_s256_burn.txt
