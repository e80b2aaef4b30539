#!/bin/bash
# tools/ab_bench_phases.sh ROUNDS [bench args] -- alternate bench runs over the
# A/B libraries (_build/ab/lib*.so) with the untimed FIR-phase legs on (no
# parity / CPU / framer / host-ring legs): value, kernel ms, FIR-alone ms and
# the FIR phase sample (free vs loop-shared CUs, pipelined).
set -e
rounds=$1; shift
for i in $(seq 1 "$rounds"); do
  for lib in qpsk-modulator-demodulator_amd/_build/ab/lib*.so; do
    QPSK_DEMOD_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-parity --no-cpu-baseline --no-framer \
          --no-host-ring --sub-configs none --detail /tmp/ab_phases_detail.json "$@" > /dev/null
    echo "$(basename "$lib") $(python3 -c '
import json
d = json.load(open("/tmp/ab_phases_detail.json")); r = d["rooflines"]
ph = r["fir"].get("phases", {}).get("pipelined", {})
print(d["value"], {k: round(v["ms"], 2) for k, v in r.items()},
      {c: (ph[c]["workgroups"], ph[c]["stage"], ph[c]["compute"], ph[c]["store"]) for c in ph})')"
  done
done
