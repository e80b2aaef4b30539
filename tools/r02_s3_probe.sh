#!/bin/bash
# stamped loop-kernel probes (tools/loop_probe.hip): A = previous kernel, B = working tree
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}; O=$R/gpurun_out; mkdir -p $O; cd $R
( for i in 1 2; do
  for b in A B; do echo "== $b C3"; timeout -k 10 60 tools/bin/loop_probe_$b 4096 1048576 0 0 0 4 | grep -v "^ WG  *[0-9]*:" || exit 1; done
  for b in A B; do echo "== $b C2"; timeout -k 10 60 tools/bin/loop_probe_$b 256 1048576 0 0 0 8 | grep -v "^ WG  *[0-9]*:" || exit 1; done
  done ) > $O/s3_probe.log 2>&1
cat $O/s3_probe.log
