#!/bin/bash
# 12 streams x 256-sample rounds (loop_variant 5, sps >= 8) vs the C2 auto
# shape 24 x 128: parity, C2 bench A/B, stamped probe.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -q -x -k "chunked_ragged" --timeout 200 --timeout-method thread > $O/v12_test.log 2>&1 || { tail -30 $O/v12_test.log; exit 1; }
tail -1 $O/v12_test.log
for i in 1 2 3; do
  for v in 4 5; do
    out=$(timeout -k 10 300 python3 bench.py --timed-only --config c2 --steps 8 --warmup 2 --loop-variant $v) || exit 1
    echo "c2 v$v $(echo "$out" | grep -o '"loop": [0-9][0-9.]*' | head -1) $(echo "$out" | grep -o '"value": [0-9.]*' | head -1)"
  done
done
for v in 4 5; do echo "== probe v$v"; timeout -k 10 60 tools/bin/loop_probe 256 1048576 $v 0 0 8 | grep -v "^ WG  *[0-9]*:" | cut -c1-400 || exit 1; done
