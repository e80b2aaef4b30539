#!/bin/bash
# A/B of the FIR work-sharing variants (QPSK_FIR_SHARE) at C3, pipelined bench.
# GPU suite first with the variant under test, then alternating bench runs.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
V=${1:-6256}
QPSK_FIR_SHARE=$V timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/ab_share_tests_$V.log" 2>&1
echo "tests ok ($V)"
for m in 0 $V 4256 0 $V 4128 8256; do
  QPSK_FIR_SHARE=$m timeout -k 10 200 python bench.py --config c3 --sub-configs none --no-cpu-baseline \
    --no-framer --no-host-ring --steps 10 --warmup 2 > "$O/ab_share_$m.json" 2> "$O/ab_share_$m.err"
  python - "$O/ab_share_$m.json" $m <<'PY' | tee -a "$O/ab_share_summary.txt"
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
p = d["parity_vs_portable_oracle"]
print(f"mode {sys.argv[2]:>5}: {d['value']:9.1f} MSa/s  step {d['ms_per_step']:.2f} ms  "
      f"fir {d['stages_ms']['fir']:.2f} loop {d['stages_ms']['loop']:.2f}  parity bits {p['bit_mismatch_streams']} syms {p['symbol_mismatch_streams']}")
PY
done
