#!/bin/bash
# tools/ab_env.sh ROUNDS "ENV=V ..." "ENV=V ..." -- [bench args]: alternate
# bench.py runs of the in-tree build under environment variants on one box
set -e
rounds=$1; shift
variants=()
while [ "$1" != "--" ]; do variants+=("$1"); shift; done
shift
for i in $(seq 1 "$rounds"); do
  for v in "${variants[@]}"; do
    out=$(env $v timeout -k 10 300 python bench.py --timed-only "$@")
    echo "[$v] $(echo "$out" | grep -o '"fir": [0-9.]*' | head -1) $(echo "$out" | grep -o '"loop": [0-9.]*' | head -1) $(echo "$out" | grep -o '"value": [0-9.]*' | head -1)"
  done
done
