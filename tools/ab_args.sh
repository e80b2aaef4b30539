#!/bin/bash
# tools/ab_args.sh ROUNDS "ARGS A" "ARGS B" ... -- [common bench args]: alternate
# bench.py --timed-only runs of the in-tree build over argument variants on one
# box (e.g. --loop-variant 0 vs 6).  Prints per run: kernel ms, the loop's
# cycles per symbol and median clock, value.
set -e
rounds=$1; shift
variants=()
while [ "$1" != "--" ]; do variants+=("$1"); shift; done
shift
for i in $(seq 1 "$rounds"); do
  for v in "${variants[@]}"; do
    out=$(timeout -k 10 300 python bench.py --timed-only $v "$@" 2> /dev/null | tail -1)
    echo "[$v] $(echo "$out" | python3 -c '
import json, sys
d = json.loads(sys.stdin.read())
r = d["kernels"]
ms = {k: round(v["ms"], 2) for k, v in r.items() if isinstance(v, dict) and "ms" in v}
lp = r.get("loop", {})
print(ms, "loop cyc/sym", lp.get("cycles_per_symbol"), "GHz", lp.get("clock_ghz_median"), "value", d["value"])')"
  done
done
