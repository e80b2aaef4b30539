#!/bin/bash
# LDS-footprint diagnostic (round 6): the loop workgroup padded by 10 / 20 KB
# (-DQPSK_LDS_PAD, 32 x 64 shapes only) so fewer FIR workgroups fit beside it
set -e -o pipefail
mkdir -p gpurun_out/ldspad
for c in c3 c4; do
  timeout -k 10 900 bash tools/ab_bench.sh 2 --config $c --steps 10 --warmup 3 2>&1 | tee -a gpurun_out/ldspad/ab_$c.txt
done
