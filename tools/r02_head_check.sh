#!/bin/bash
# HEAD re-check: GPU suite, smoke, default bench, rocprofv3 stats of the C3 timed region.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > "$O/head_gputest.log" 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$O/head_smoke.log" 2>&1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > "$O/head_bench.json" 2> "$O/head_bench.err"
echo "bench done"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/head_prof_c3" -o run \
  -- python3 "$R/bench.py" --config c3 --steps 20 --warmup 5 --timed-only > "$O/head_prof_c3.log" 2>&1
echo "profiled"
