#!/bin/bash
# tools/ab_bench.sh -- alternate bench.py runs over in-tree library builds
# (qpsk-modulator-demodulator_amd/_build/ab/lib*.so) on one box, so kernel
# variants are compared under the same clocks.  Usage: tools/ab_bench.sh ROUNDS [bench args]
# Prints per run: kernel ms, the loop's cycles per symbol and median clock, value.
set -e
rounds=$1; shift
for i in $(seq 1 "$rounds"); do
  for lib in qpsk-modulator-demodulator_amd/_build/ab/lib*.so; do
    out=$(QPSK_DEMOD_LIB=$PWD/$lib timeout -k 10 300 python bench.py --timed-only "$@" 2> /dev/null | tail -1)
    echo "$(basename "$lib") $(echo "$out" | python3 -c '
import json, sys
d = json.loads(sys.stdin.read())
r = d["kernels"]
ms = {k: round(v["ms"], 2) for k, v in r.items() if isinstance(v, dict) and "ms" in v}
lp = r.get("loop", {})
print(ms, "loop cyc/sym", lp.get("cycles_per_symbol"), "GHz", lp.get("clock_ghz_median"), "value", d["value"])')"
  done
done
