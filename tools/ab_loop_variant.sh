#!/bin/bash
# tools/ab_loop_variant.sh ROUNDS CONFIG V1 V2 ...: alternate bench.py --timed-only
# runs of loop shapes (qpsk_demod_params.loop_variant) on one box
set -e
rounds=$1; cfg=$2; shift 2
for i in $(seq 1 "$rounds"); do
  for v in "$@"; do
    out=$(timeout -k 10 300 python bench.py --timed-only --config "$cfg" --loop-variant "$v" --steps 10 --warmup 3 2>/dev/null | tail -1)
    echo "[variant $v] $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d.get("kernels",{}); print("value", d["value"], "stages_ms", json.dumps(d.get("stages_ms")), "loop_cps", k.get("loop",{}).get("cycles_per_symbol"))')"
  done
done
