#!/bin/bash
# final state of the round: GPU suite, smoke(), the driver's default bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/final_gputest.log 2>&1 || { tail -30 $O/final_gputest.log; exit 1; }
tail -2 $O/final_gputest.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/final_smoke.log 2>&1 || { tail -20 $O/final_smoke.log; exit 1; }
tail -1 $O/final_smoke.log
timeout -k 10 500 python3 bench.py > $O/final_bench.json 2> $O/final_bench.err || { tail -20 $O/final_bench.err; exit 1; }
python3 -c "
import json; r=json.load(open('$O/final_bench.json'))
print('C3', r['value'], r['ms_per_step'], r['stages_ms'], r['parity_vs_libm_oracle']['mismatching_streams'], r['roofline'])
for k,v in r['sub_records'].items(): print(k, v['value'], v['ms_per_step'], v['stages_ms'], v['parity_vs_libm_oracle']['mismatching_streams'])
"
