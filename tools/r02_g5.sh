set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/r02_gputest2.log 2>&1 || exit 1
timeout -k 10 600 python3 bench.py > $O/r02_bench_default2.json 2> $O/r02_bench_default2.err || exit 1
