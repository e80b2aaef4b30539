#!/bin/bash
# Round-2 evidence of the current build (committed under profiles/ by hand):
#   1. rocprofv3 --kernel-trace --stats of the bench's timed region, C3/C2/C5
#   2. FIR HBM traffic at C3 (separate FETCH_SIZE / WRITE_SIZE passes)
#   3. per-dispatch clock at C3 (GRBM_GUI_ACTIVE, dispatches serialised)
#   4. stamped loop probe: C2 (24 x 128 and 32 x 64), C3
#   5. 2-rank gloo rehearsal of the C4 shard shape on this one GPU
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
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$O/r02_c3_grbm" -o run \
  -- python3 "$R/bench.py" --config c3 --steps 6 --warmup 2 --timed-only > "$O/r02_c3_grbm.log" 2>&1
python3 "$R/tools/dispatch_clock.py" "$O/r02_c3_grbm" --out "$O/r02_c3_grbm_clock.json" \
  --what "C3 bench --timed-only under rocprofv3 --pmc GRBM_GUI_ACTIVE (dispatches serialised), round-2 final build; effective clock = GRBM_GUI_ACTIVE / 8 / wall"
echo "clock done"
cd "$R"
( echo "== C2 24x128 (variant 4, the C2 auto shape)"; timeout -k 10 60 tools/bin/loop_probe 256 1048576 4 0 0 8 | grep -v "^ WG  *[0-9]*:"
  echo "== C2 32x64 (variant 2)"; timeout -k 10 60 tools/bin/loop_probe 256 1048576 2 0 0 8 | grep -v "^ WG  *[0-9]*:"
  echo "== C3 32x64 (auto)"; timeout -k 10 60 tools/bin/loop_probe 4096 1048576 0 0 0 4 | grep -v "^ WG  *[0-9]*:" ) > "$O/r02_loop_probe_final.log" 2>&1
echo "probe done"
timeout -k 10 600 python3 bench.py --gpus 2 --dist-backend gloo --share-gpu --config c4 --streams 1024 --steps 3 --warmup 1 \
  --no-cpu-baseline > "$O/r02_c4_2rank_gloo_rehearsal.json" 2> "$O/r02_c4_2rank_gloo_rehearsal.err"
echo "rehearsal done"
