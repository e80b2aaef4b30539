#!/bin/bash
# tools/ab_env.sh ROUNDS "ENV=V ..." "ENV=V ..." -- [bench args]: alternate
# bench.py runs of the in-tree build under environment variants on one box;
# prints each run's value, stage times and the loop's cycles per symbol
set -e
rounds=$1; shift
variants=()
while [ "$1" != "--" ]; do variants+=("$1"); shift; done
shift
for i in $(seq 1 "$rounds"); do
  for v in "${variants[@]}"; do
    out=$(env $v timeout -k 10 300 python bench.py --timed-only "$@" 2>/dev/null | tail -1)
    echo "[$v] $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d.get("kernels",{}); print("value", d["value"], "stages_ms", json.dumps(d.get("stages_ms")), "loop_cps", k.get("loop",{}).get("cycles_per_symbol"))')"
  done
done
