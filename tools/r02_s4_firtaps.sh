#!/bin/bash
# FIR taps phase-major (B: one s_load_dwordx16 per lane phase) against the
# strided copy (A: 16 s_load_dword interleaved with the LDS reads, each use
# behind an lgkmcnt(0) that also waits for them).  GPU suite on B, then A/B x2.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | tail -2 || exit 1
L=qpsk-modulator-demodulator_amd/_build/ab
run() { out=$(QPSK_DEMOD_LIB=$PWD/$L/lib$1.so timeout -k 10 300 python3 bench.py --timed-only --config $2 --steps $3 --warmup 2 $4) || exit 1
  echo "$2 $4 lib$1 $(echo "$out" | grep -o '"fir": [0-9][0-9.]*' | head -1) $(echo "$out" | grep -o '"loop": [0-9][0-9.]*' | head -1) $(echo "$out" | grep -o '"ms_per_step": [0-9.]*' | head -1) $(echo "$out" | grep -o '"value": [0-9.]*' | head -1)"; }
for i in 1 2; do
  for l in A B; do run $l c3 8; done
  for l in A B; do run $l c3 4 --serial-calls; done
  for l in A B; do run $l c2 8 --serial-calls; done
done
