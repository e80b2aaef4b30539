#!/bin/bash
# GPU suite + the driver's default bench on the current tree
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/s3b_gputest.log 2>&1 || { tail -30 $O/s3b_gputest.log; exit 1; }
tail -2 $O/s3b_gputest.log
timeout -k 10 500 python3 bench.py > $O/s3b_bench.json 2> $O/s3b_bench.err || { tail -20 $O/s3b_bench.err; exit 1; }
python3 -c "
import json; r=json.load(open('$O/s3b_bench.json'))
print('C3', r['value'], r['ms_per_step'], r['stages_ms'], r['parity_vs_libm_oracle']['mismatching_streams'])
for k,v in r['sub_records'].items(): print(k, v['value'], v['ms_per_step'], v['stages_ms'], v['parity_vs_libm_oracle']['mismatching_streams'])
"
