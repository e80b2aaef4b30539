#!/bin/bash
# 24 streams x 128-sample rounds (loop_variant 4, sps >= 8) vs the default
# 32 x 64: GPU suite, then C2 (and C5 serial) loop-stage A/B on one box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python3 -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/v4_test.log 2>&1 || { tail -30 $O/v4_test.log; exit 1; }
tail -1 $O/v4_test.log
for i in 1 2 3; do
  for v in 0 4; do
    out=$(timeout -k 10 300 python3 bench.py --timed-only --config c2 --steps 8 --warmup 2 --loop-variant $v) || exit 1
    echo "c2 v$v $(echo "$out" | grep -o '"loop": [0-9][0-9.]*' | head -1) $(echo "$out" | grep -o '"value": [0-9.]*' | head -1)"
  done
done
for v in 0 4; do
  out=$(timeout -k 10 300 python3 bench.py --timed-only --config c5 --steps 3 --warmup 1 --serial-calls --loop-variant $v) || exit 1
  echo "c5 serial v$v $(echo "$out" | grep -o '"loop": [0-9][0-9.]*' | head -1) $(echo "$out" | grep -o '"value": [0-9.]*' | head -1)"
done
