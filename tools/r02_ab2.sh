set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/r02_gputest4.log 2>&1 || exit 1
for c in c2 c3; do echo "== $c"; timeout -k 10 500 bash tools/ab_bench.sh 3 --config $c --steps 8 --warmup 2 || exit 1; done > $O/r02_ab2.log 2>&1
echo "== c2 variant 3" >> $O/r02_ab2.log
QPSK_DEMOD_LIB=$R/qpsk-modulator-demodulator_amd/_build/ab/libB_costas.so timeout -k 10 200 python3 bench.py --timed-only --config c2 --steps 8 --loop-variant 3 >> $O/r02_ab2.log 2>&1
