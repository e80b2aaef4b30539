#!/bin/bash
# tools/gpu_profile.sh ROUND CONFIG -- rocprofv3 evidence for bench.py's roofline.
#   1. --kernel-trace --stats of the bench's warmup + timed steps only
#      (--timed-only), so the kernel averages are the timed region's
#      -> gpurun_out/prof_<round>_<cfg>/
#   2. separate --pmc FETCH_SIZE and WRITE_SIZE passes (never combined with
#      trace domains) -> tools/pmc_traffic.py -> profiles/pmc_fir_<cfg>.json
# Run on the GPU box via gpurun; every GPU step has its own time limit.
set -e -o pipefail
ROUND=${1:-r01}
CFG=${2:-c2}
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p "$O" "$R/profiles"
cd /tmp && export TMPDIR=/tmp
case "$CFG" in
  c2) ALGO=$((256 * 1048576 * 16)) ;;
  c3|c4) ALGO=$((4096 * 1048576 * 16)) ;;
  c5) ALGO=$((8192 * 1048576 * 16)) ;;
esac
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_${ROUND}_${CFG}" -o run \
  -- python3 "$R/bench.py" --config "$CFG" --steps 6 --warmup 2 --timed-only > "$O/prof_${ROUND}_${CFG}.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_fetch_${CFG}" -o run \
  -- python3 "$R/bench.py" --config "$CFG" --steps 2 --warmup 1 --no-cpu-baseline --no-parity > "$O/pmc_fetch_${CFG}.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_write_${CFG}" -o run \
  -- python3 "$R/bench.py" --config "$CFG" --steps 2 --warmup 1 --no-cpu-baseline --no-parity > "$O/pmc_write_${CFG}.log" 2>&1
python3 "$R/tools/pmc_traffic.py" --fetch "$O/pmc_fetch_${CFG}" --write "$O/pmc_write_${CFG}" \
  --kernel fir_tile_kernel --algo-bytes "$ALGO" --out "$O/pmc_fir_${CFG}.json"
