#!/bin/bash
# float M&M -> Costas slots (round 6) against double slots, every shape
set -e -o pipefail
mkdir -p gpurun_out/fslots2
for c in c2 c4 c3; do
  timeout -k 10 900 bash tools/ab_bench.sh 2 --config $c --steps 10 --warmup 3 2>&1 | tee -a gpurun_out/fslots2/ab_$c.txt
done
for L in base fsall; do
  QPSK_DEMOD_LIB=$PWD/qpsk-modulator-demodulator_amd/_build/ab/lib$L.so timeout -k 10 600 python bench.py --config c3 --sub-configs none --no-drop-in --no-host-ring --no-framer --no-cpu-baseline --no-parity --steps 10 --warmup 3 --detail gpurun_out/fslots2/detail_$L.json > gpurun_out/fslots2/line_$L.json 2>/dev/null
done
