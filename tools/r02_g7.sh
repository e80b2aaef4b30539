set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r02_gputest5.log 2>&1 || exit 1
( for b in A E; do echo "== $b C2"; timeout -k 10 60 tools/bin/loop_probe_$b 256 1048576 0 0 0 8 | grep -v "^ WG  *[0-9]*:" || exit 1; done
  echo "== E C2 v3"; timeout -k 10 60 tools/bin/loop_probe_E 256 1048576 3 0 0 8 || exit 1
  for b in A E; do echo "== $b C3"; timeout -k 10 60 tools/bin/loop_probe_$b 4096 1048576 0 0 0 4 | grep -v "^ WG  *[0-9]*:" || exit 1; done ) > $O/r02_probe3.log 2>&1 || exit 1
for c in c2 c3; do echo "== $c"; timeout -k 10 500 bash tools/ab_bench.sh 2 --config $c --steps 8 --warmup 2 || exit 1; done > $O/r02_ab3.log 2>&1
