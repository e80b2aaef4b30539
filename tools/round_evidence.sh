#!/bin/bash
# tools/round_evidence.sh ROUND -- the evidence a round commits under profiles/:
# rocprofv3 kernel stats + FIR PMC traffic for C2/C3 (tools/gpu_profile.sh),
# then the bench line of C2 (headline), C3 and C5 with the CPU baseline.
# Every GPU step has its own time limit; the script stops at the first failure.
set -e -o pipefail
ROUND=${1:-r01}
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out
mkdir -p "$O"
for c in c2 c3; do
  bash "$R/tools/gpu_profile.sh" "$ROUND" "$c"
  echo "profiled $c"
done
for c in c2 c3 c5; do
  timeout -k 10 300 python3 "$R/bench.py" --config "$c" --steps 6 --warmup 2 > "$O/${ROUND}_${c}_bench.json" 2> "$O/${ROUND}_${c}_bench.err"
  echo "bench $c"; cat "$O/${ROUND}_${c}_bench.json"
done
