#!/bin/bash
# Shadow lanes (lanes past a workgroup's streams run its first stream's
# chains): the lane-count probe again, the GPU suite, then C2 / small-batch
# bench A/B (A = without shadows).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}; O=$R/gpurun_out; mkdir -p $O; cd $R
for s in 1 8 16 24 32; do
  timeout -k 10 120 tools/bin/loop_probe $s 1048576 2 0 0 8.0 > $O/probe_shadow$s.txt 2>&1 || exit 1
  echo "S=$s $(head -1 $O/probe_shadow$s.txt | grep -o '[0-9.]* ms') $(grep 'rounds' $O/probe_shadow$s.txt | head -1 | grep -o 'cyc/sym.*')"
done
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | tail -3 || exit 1
L=qpsk-modulator-demodulator_amd/_build/ab
run() { out=$(QPSK_DEMOD_LIB=$PWD/$L/lib$1.so timeout -k 10 300 python3 bench.py --timed-only --config $2 --steps $3 --warmup 2 $4) || exit 1
  echo "$2 $4 lib$1 $(echo "$out" | grep -o '"loop": [0-9][0-9.]*' | head -1) $(echo "$out" | grep -o '"ms_per_step": [0-9.]*' | head -1) $(echo "$out" | grep -o '"value": [0-9.]*' | head -1)"; }
for i in 1 2; do
  for l in A B; do run $l c2 8 "--streams 1"; done
  for l in A B; do run $l c2 8 "--streams 40"; done
  for l in A B; do run $l c2 8; done
done
