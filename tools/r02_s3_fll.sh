#!/bin/bash
# FLL register-window blocks + bit-op quadrant logic: GPU suite, then A/B of the
# C5 chain (pipelined and serial calls) against the previous FLL build.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python3 -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/fll_test.log 2>&1 || { tail -30 $O/fll_test.log; exit 1; }
tail -1 $O/fll_test.log
for i in 1 2; do
  for lib in qpsk-modulator-demodulator_amd/_build/ab/lib*.so; do
    for mode in "" "--serial-calls"; do
      out=$(QPSK_DEMOD_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --timed-only --config c5 --steps 4 --warmup 1 $mode) || exit 1
      echo "$(basename $lib) ${mode:-pipelined} $(echo "$out" | grep -o '"fll": [0-9][0-9.]*' | head -1) $(echo "$out" | grep -o '"loop": [0-9][0-9.]*' | head -1) $(echo "$out" | grep -o '"value": [0-9.]*' | head -1)"
    done
  done
done
