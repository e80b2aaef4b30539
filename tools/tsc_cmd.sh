set -e -o pipefail
mkdir -p gpurun_out/tsc1
timeout -k 10 300 python -u -m pytest tests/test_framer.py tests/test_gpu_parity.py -k "framer or tsc or c_abi_demo or bytes_chain" -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/tsc1/test.log 2>&1 || { tail -30 gpurun_out/tsc1/test.log; exit 1; }
tail -2 gpurun_out/tsc1/test.log
for c in c2 c3; do timeout -k 10 200 python tools/framer_bench.py --config $c --reps 10 2>>gpurun_out/tsc1/err.log | tail -1 | tee -a gpurun_out/tsc1/bench.jsonl; done
