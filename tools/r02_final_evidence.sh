#!/bin/bash
# Round-2 evidence of the final build (copied into profiles/ by hand):
#   1. GPU suite, smoke
#   2. rocprofv3 --kernel-trace --stats of the bench's timed region, C3/C2/C5
#   3. FIR HBM traffic at C3 (separate FETCH_SIZE / WRITE_SIZE passes)
#   4. the default bench line
# Every GPU step has its own time limit; the script stops at the first failure.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > "$O/fin_gputest.log" 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$O/fin_smoke.log" 2>&1
echo "tests ok"
cd /tmp && export TMPDIR=/tmp
for c in c3 c2 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/fin_prof_$c" -o run \
    -- python3 "$R/bench.py" --config $c --steps 10 --warmup 2 --timed-only > "$O/fin_prof_$c.log" 2>&1
  echo "profiled $c"
done
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/fin_pmc_fetch_c3" -o run \
  -- python3 "$R/bench.py" --config c3 --steps 2 --warmup 1 --timed-only > "$O/fin_pmc_fetch_c3.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/fin_pmc_write_c3" -o run \
  -- python3 "$R/bench.py" --config c3 --steps 2 --warmup 1 --timed-only > "$O/fin_pmc_write_c3.log" 2>&1
python3 "$R/tools/pmc_traffic.py" --fetch "$O/fin_pmc_fetch_c3" --write "$O/fin_pmc_write_c3" \
  --kernel fir_tile_kernel --algo-bytes $((4096 * 1048576 * 16)) --out "$O/fin_pmc_fir_c3.json"
echo "pmc done"
cd "$R"
timeout -k 10 400 python bench.py > "$O/fin_bench.json" 2> "$O/fin_bench.err"
echo "bench done"
