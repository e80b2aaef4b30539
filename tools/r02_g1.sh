set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
( python3 -c "import os; print('cpu_count', os.cpu_count(), 'affinity', len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max 2>&1; nproc; lscpu | head -20 ) > $O/box_cpu.txt 2>&1
cd $R && timeout -k 10 300 python3 bench.py --config c3 --steps 10 --warmup 2 --no-host-ring > $O/r02_c3_base.json 2> $O/r02_c3_base.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/r02_c3_grbm -o run -- python3 $R/bench.py --config c3 --steps 10 --warmup 2 --timed-only > $O/r02_c3_grbm.log 2>&1
