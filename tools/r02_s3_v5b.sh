#!/bin/bash
# 40 streams x 64-sample rounds with byte decisions (loop_variant 5): every lane of the stage waves
# busy, half the loop's VALU work per stream, twice its round bookkeeping per
# symbol.  Parity of the new shape, then C3 A/B against the auto shape.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -q -x -k "chunked_ragged or huge or nonfinite or constellation or nondifferential" --timeout 200 --timeout-method thread > $O/v5b_test.log 2>&1 || { tail -30 $O/v5b_test.log; exit 1; }
tail -1 $O/v5b_test.log
for i in 1 2; do
  for v in 0 5; do
    for mode in "" "--serial-calls"; do
      out=$(timeout -k 10 300 python3 bench.py --timed-only --config c3 --steps 8 --warmup 2 --loop-variant $v $mode) || exit 1
      echo "c3 v$v ${mode:-pipelined} $(echo "$out" | grep -o '"fir": [0-9][0-9.]*' | head -1) $(echo "$out" | grep -o '"loop": [0-9][0-9.]*' | head -1) $(echo "$out" | grep -o '"value": [0-9.]*' | head -1)"
    done
  done
done
