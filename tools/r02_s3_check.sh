#!/bin/bash
# re-entry check: GPU suite + the driver's default bench on the restored tree
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/s3_gputest.log 2>&1 || { tail -30 $O/s3_gputest.log; exit 1; }
tail -3 $O/s3_gputest.log
timeout -k 10 400 python3 bench.py > $O/s3_bench.json 2> $O/s3_bench.err || { tail -20 $O/s3_bench.err; exit 1; }
cat $O/s3_bench.json
