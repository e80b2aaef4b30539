set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
( for b in A B; do echo "== $b C2 v0"; timeout -k 10 60 tools/bin/loop_probe_$b 256 1048576 0 || exit 1; done
  echo "== B C2 v3"; timeout -k 10 60 tools/bin/loop_probe_B 256 1048576 3 0 0 8 || exit 1
  echo "== B C3 v0"; timeout -k 10 60 tools/bin/loop_probe_B 4096 1048576 0 0 0 4 || exit 1 ) > $O/r02_probe1.log 2>&1
