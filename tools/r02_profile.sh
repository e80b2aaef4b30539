#!/bin/bash
# round-2 rocprofv3 evidence: kernel stats of the bench's timed region for
# C3 (headline), C2, C5; FIR PMC traffic at C3; per-dispatch clock at C3.
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
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$O/r02_c3_grbm" -o run \
  -- python3 "$R/bench.py" --config c3 --steps 10 --warmup 2 --timed-only > "$O/r02_c3_grbm.log" 2>&1
python3 "$R/tools/dispatch_clock.py" "$O/r02_c3_grbm" --out "$O/r02_c3_grbm_clock.json" \
  --what "C3 bench --timed-only under rocprofv3 --pmc GRBM_GUI_ACTIVE (dispatches serialised), round-2 build; effective clock = GRBM_GUI_ACTIVE / 8 / wall"
