set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 600 python3 bench.py > $O/r02_bench_default.json 2> $O/r02_bench_default.err || exit 1
timeout -k 10 300 python3 bench.py --gpus 2 --dist-backend gloo --share-gpu --streams 256 --steps 3 --sub-configs c4 --cpu-seconds 2 > $O/r02_bench_2rank.json 2> $O/r02_bench_2rank.err || exit 1
