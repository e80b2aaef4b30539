#!/bin/bash
# tools/ab_bench_fll.sh ROUNDS [bench args] -- alternate timed-only bench runs
# over the A/B libraries (_build/ab/lib*.so), printing each kernel's launch ms
# and the value; diagnostic variants' results are wrong by design.
set -e
rounds=$1; shift
for i in $(seq 1 "$rounds"); do
  for lib in qpsk-modulator-demodulator_amd/_build/ab/lib*.so; do
    out=$(QPSK_DEMOD_LIB=$PWD/$lib timeout -k 10 300 python bench.py --timed-only "$@")
    echo "$(basename "$lib") $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["kernels"]; print({k: round(v["ms"], 2) for k, v in r.items()}, {k: r[k].get("cycles_per_sample") for k in r if "cycles_per_sample" in r[k]}, d["value"])')"
  done
done
