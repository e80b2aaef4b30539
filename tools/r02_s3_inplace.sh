#!/bin/bash
# Costas in place (double slots, range bound instead of per-symbol tracking):
# GPU suite, then C3 / C2 A/B against the previous loop kernel on one box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python3 -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/inplace_test.log 2>&1 || { tail -30 $O/inplace_test.log; exit 1; }
tail -1 $O/inplace_test.log
for i in 1 2; do
  for c in c3 c2; do
    for lib in qpsk-modulator-demodulator_amd/_build/ab/lib*.so; do
      for mode in "" "--serial-calls"; do
        out=$(QPSK_DEMOD_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --timed-only --config $c --steps 6 --warmup 2 $mode) || exit 1
        echo "$c $(basename $lib) ${mode:-pipelined} $(echo "$out" | grep -o '"fir": [0-9][0-9.]*' | head -1) $(echo "$out" | grep -o '"loop": [0-9][0-9.]*' | head -1) $(echo "$out" | grep -o '"value": [0-9.]*' | head -1)"
      done
    done
  done
done
