#!/bin/bash
# Streams spread evenly over the loop workgroups (B) against blocks of SPW
# with a partly filled last one (A): stamped probe, then C2 / C3 / C4-shard
# bench A/B x2, then the GPU suite on B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}; O=$R/gpurun_out; mkdir -p $O; cd $R
for s in 256 4096; do
  timeout -k 10 120 tools/bin/loop_probe $s 1048576 4 0 0 8.0 > $O/probe_even$s.txt 2>&1 || exit 1
  head -1 $O/probe_even$s.txt; grep -E "^ WG +[0-9]+:" $O/probe_even$s.txt | sed 's/.*| M&M //' | sort | uniq -c | sort -rn | head -3
done
L=qpsk-modulator-demodulator_amd/_build/ab
run() { out=$(QPSK_DEMOD_LIB=$PWD/$L/lib$1.so timeout -k 10 300 python3 bench.py --timed-only --config $2 --steps $3 --warmup 2 $4) || exit 1
  echo "$2 $4 lib$1 $(echo "$out" | grep -o '"fir": [0-9][0-9.]*' | head -1) $(echo "$out" | grep -o '"loop": [0-9][0-9.]*' | head -1) $(echo "$out" | grep -o '"ms_per_step": [0-9.]*' | head -1) $(echo "$out" | grep -o '"value": [0-9.]*' | head -1)"; }
for i in 1 2; do
  for l in A B; do run $l c2 10; done
  for l in A B; do run $l c4 4 "--streams 4096"; done
  for l in A B; do run $l c3 6; done
done
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | tail -3
