set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04d
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for c in c3 c2 c5; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$c -o run -- python3 $R/bench.py --config $c --steps 10 --warmup 2 --timed-only > $O/prof_$c.log 2>&1
  echo "prof $c done"
done
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_c2 -o run -- python3 $R/bench.py --config c2 --steps 2 --warmup 1 --no-cpu-baseline --no-parity > $O/pmc_fetch_c2.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_c2 -o run -- python3 $R/bench.py --config c2 --steps 2 --warmup 1 --no-cpu-baseline --no-parity > $O/pmc_write_c2.log 2>&1
python3 $R/tools/pmc_traffic.py --fetch $O/pmc_fetch_c2 --write $O/pmc_write_c2 --kernel loop_kernel --algo-bytes 2155872256 --out $O/pmc_loop_c2.json
echo all done
