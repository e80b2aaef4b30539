set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
( python3 -c "import os; print('cpu_count', os.cpu_count(), 'affinity', len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max 2>&1; nproc; lscpu | head -20 ) > $O/box_cpu.txt 2>&1
cd $R && timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r02_gputest.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --config c3 --steps 10 --warmup 2 --no-host-ring --no-cpu-baseline > $O/r02_c3_after.json 2> $O/r02_c3_after.err || exit 1
timeout -k 10 240 python3 tools/state_probe.py --config c3 --calls 14 > $O/r02_state_c3_after.log 2>&1
