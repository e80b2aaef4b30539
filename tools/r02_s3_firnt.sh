#!/bin/bash
# A/B: FIR workgroup size (QPSK_FIR_THREADS = 256 / 128 / 64 threads = 2048 /
# 1024 / 512 outputs per tile) at C3 and C2, pipelined bench, same box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}; O=$R/gpurun_out; mkdir -p $O; cd $R
for nt in 128 64; do
  QPSK_FIR_THREADS=$nt timeout -k 10 300 python3 -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/firnt_test_$nt.log 2>&1 || { echo "tests failed nt=$nt"; tail -20 $O/firnt_test_$nt.log; exit 1; }
  tail -1 $O/firnt_test_$nt.log
done
for i in 1 2; do
  for c in c3 c2; do
    for nt in 256 128 64; do
      out=$(QPSK_FIR_THREADS=$nt timeout -k 10 300 python3 bench.py --timed-only --config $c --steps 8 --warmup 2) || exit 1
      echo "$c nt=$nt $(echo "$out" | grep -o '"fir": [0-9.]*') $(echo "$out" | grep -o '"loop": [0-9.]*') $(echo "$out" | grep -o '"value": [0-9.]*')"
    done
  done
done
