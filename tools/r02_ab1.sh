set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
for c in c3 c2 c5; do echo "== $c"; timeout -k 10 500 bash tools/ab_bench.sh 2 --config $c --steps 8 --warmup 2 || exit 1; done > $O/r02_ab1.log 2>&1
