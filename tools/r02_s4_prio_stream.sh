#!/bin/bash
# Stream priority with the FLL on: A = back stream (FIR + loop) first (old),
# B = front waits only for the FIR + loop waves at s_setprio 3, C = FIR wait only,
# D = priority only.  C5 pipelined bench, x2.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}; O=$R/gpurun_out; mkdir -p $O; cd $R
L=qpsk-modulator-demodulator_amd/_build/ab
run() { out=$(QPSK_DEMOD_LIB=$PWD/$L/lib$1.so timeout -k 10 300 python3 bench.py --timed-only --config $2 --steps $3 --warmup 2) || exit 1
  echo "$2 lib$1 $(echo "$out" | grep -o '"fll": [0-9][0-9.]*' | head -1) $(echo "$out" | grep -o '"fir": [0-9][0-9.]*' | head -1) $(echo "$out" | grep -o '"loop": [0-9][0-9.]*' | head -1) $(echo "$out" | grep -o '"ms_per_step": [0-9.]*' | head -1) $(echo "$out" | grep -o '"value": [0-9.]*' | head -1)"; }
for i in 1 2; do
  for l in A B C D; do run $l c5 6; done
done
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "fll or pipelin or async" 2>&1 | tail -5
