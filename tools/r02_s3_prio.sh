#!/bin/bash
# Wave priority (s_setprio) A/B: A = none, B = FIR at prio 2, C = FLL at 2,
# D = FIR 2 + FLL 3.  VALU issue goes by priority, then age; the long-lived
# loop/FLL waves are older than the FIR's, so today they win every tie.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}; O=$R/gpurun_out; mkdir -p $O; cd $R
L=qpsk-modulator-demodulator_amd/_build/ab
run() { out=$(QPSK_DEMOD_LIB=$PWD/$L/lib$1.so timeout -k 10 300 python3 bench.py --timed-only --config $2 --steps $3 --warmup 2) || exit 1
  echo "$2 lib$1 $(echo "$out" | grep -o '"fll": [0-9][0-9.]*' | head -1) $(echo "$out" | grep -o '"fir": [0-9][0-9.]*' | head -1) $(echo "$out" | grep -o '"loop": [0-9][0-9.]*' | head -1) $(echo "$out" | grep -o '"value": [0-9.]*' | head -1)"; }
for i in 1 2; do
  for l in A B D; do run $l c3 8; done
  for l in A C D; do run $l c5 4; done
  for l in A B; do run $l c2 8; done
done
