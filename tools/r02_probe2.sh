set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
( for b in A B C D; do echo "== $b C2"; timeout -k 10 60 tools/bin/loop_probe_$b 256 1048576 0 0 0 8 | grep -v "^ WG  *[0-9]*:" || exit 1; done
  for b in A B C D; do echo "== $b C3"; timeout -k 10 60 tools/bin/loop_probe_$b 4096 1048576 0 0 0 4 | grep -v "^ WG  *[0-9]*:" || exit 1; done ) > $O/r02_probe2.log 2>&1
