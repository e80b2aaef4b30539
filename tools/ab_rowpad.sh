#!/bin/bash
# ring rows padded by 2 samples (round 6) against the unpadded rows, C3 / C4 / C2
set -e -o pipefail
mkdir -p gpurun_out/rowpad
for c in c3 c4 c2; do
  timeout -k 10 900 bash tools/ab_bench.sh 2 --config $c --steps 10 --warmup 3 2>&1 | tee -a gpurun_out/rowpad/ab_$c.txt
done
