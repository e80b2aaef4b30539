set -e
mkdir -p gpurun_out/fr1
timeout -k 10 300 python -u -m pytest tests/test_framer.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/fr1/test.log 2>&1 || { tail -30 gpurun_out/fr1/test.log; exit 1; }
tail -2 gpurun_out/fr1/test.log
for c in c2 c3; do
  for L in base new; do
    if [ $L = base ]; then export QPSK_DEMOD_LIB=$PWD/qpsk-modulator-demodulator_amd/_build/ab/libbase.so; else unset QPSK_DEMOD_LIB; fi
    timeout -k 10 200 python tools/framer_bench.py --config $c --reps 10 2>>gpurun_out/fr1/err.log | tail -1 | tee -a gpurun_out/fr1/bench.jsonl
  done
done
