#!/bin/bash
# C3 loop shapes (round 6 re-measure): auto (32 x 64) vs 16 x 128 (variant 3)
set -e -o pipefail
mkdir -p gpurun_out/c3shapes
for i in 1 2; do
  for v in 0 3; do
    out=$(timeout -k 10 300 python bench.py --timed-only --config c3 --steps 10 --warmup 3 --loop-variant $v 2>/dev/null | tail -1)
    echo "variant $v $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernels"]; print({a:(b.get("ms"),b.get("cycles_per_symbol")) for a,b in k.items()}, "value", d["value"])')" | tee -a gpurun_out/c3shapes/ab.txt
  done
done
