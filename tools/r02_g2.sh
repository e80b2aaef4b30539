set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R && timeout -k 10 240 python3 tools/state_probe.py --config c3 --calls 14 > $O/r02_state_c3.log 2>&1
