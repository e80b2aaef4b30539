#!/bin/bash
# What in the loop kernel costs the FIR beside it?  C3 pipelined bench with
# diagnostic loop builds (results wrong, timing only): NOLOAD (no LDS DMA),
# NOMM / NOCOSTAS (stand-in waves), NODECODE (idle decode wave).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}; O=$R/gpurun_out; mkdir -p $O; cd $R
L=qpsk-modulator-demodulator_amd/_build/ab
run() { out=$(QPSK_DEMOD_LIB=$PWD/$L/lib$1.so timeout -k 10 300 python3 bench.py --timed-only --config $2 --steps $3 --warmup 2 $4) || exit 1
  echo "$2 $4 lib$1 $(echo "$out" | grep -o '"fir": [0-9][0-9.]*' | head -1) $(echo "$out" | grep -o '"loop": [0-9][0-9.]*' | head -1) $(echo "$out" | grep -o '"ms_per_step": [0-9.]*' | head -1)"; }
for i in 1 2; do
  for l in A NOLOAD NOMM NOCOSTAS NODECODE; do run $l c3 8; done
done
