#!/bin/bash
# tools/ab_probe.sh ROUNDS [loop_probe args] -- alternate the stamped loop
# probes built by tools/ab_build.sh (tools/bin/loop_probe_*) on one box:
# launch time and the per-wave cycles per symbol of the first workgroups.
set -e
rounds=$1; shift
for i in $(seq 1 "$rounds"); do
  for p in tools/bin/loop_probe_*; do
    out=$(timeout -k 10 120 "$p" "$@")
    echo "$(basename "$p") $(echo "$out" | head -1 | grep -o '[0-9.]* ms') | $(echo "$out" | grep -o 'cyc/sym M&M [0-9]* Costas [0-9]*' | head -2 | tr '\n' ' ')"
  done
done
