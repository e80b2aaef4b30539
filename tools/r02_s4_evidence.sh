#!/bin/bash
# Round-2 evidence of the current build (committed under profiles/ by hand):
#   1. rocprofv3 --kernel-trace --stats of the bench's timed region, C3/C2/C5
#   2. FIR HBM traffic at C3 (separate FETCH_SIZE / WRITE_SIZE passes)
#   3. the default bench line
# Every GPU step has its own time limit; the script stops at the first failure.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for c in c3 c2 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_r02_$c" -o run \
    -- python3 "$R/bench.py" --config $c --steps 10 --warmup 2 --timed-only > "$O/prof_r02_$c.log" 2>&1
  echo "profiled $c"
done
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_fetch_c3" -o run \
  -- python3 "$R/bench.py" --config c3 --steps 2 --warmup 1 --timed-only > "$O/pmc_fetch_c3.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_write_c3" -o run \
  -- python3 "$R/bench.py" --config c3 --steps 2 --warmup 1 --timed-only > "$O/pmc_write_c3.log" 2>&1
python3 "$R/tools/pmc_traffic.py" --fetch "$O/pmc_fetch_c3" --write "$O/pmc_write_c3" \
  --kernel fir_tile_kernel --algo-bytes $((4096 * 1048576 * 16)) --out "$O/pmc_fir_c3.json"
echo "pmc done"
cd "$R"
timeout -k 10 900 python3 -u bench.py > "$O/final_bench.json" 2> "$O/final_bench.err"
tail -c 400 "$O/final_bench.json"
