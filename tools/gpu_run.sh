#!/bin/bash
# One parametrised driver for gpurun calls (replaces round 2's one-off scripts).
#   tools/gpu_run.sh STEP [STEP ...]
# steps:
#   tests            GPU suite (-m gpu) + smoke
#   tests:EXPR       GPU suite restricted with -k EXPR
#   bench            default bench line (driver flags: --steps 20 --warmup 5)
#   bench:ARGS       bench with extra args (commas become spaces)
#   prof:CFG         rocprofv3 --kernel-trace --stats of the timed region of CFG
#   pmc:CFG:KERNEL:BYTES  FETCH_SIZE / WRITE_SIZE passes for KERNEL at CFG -> traffic json
#                    (BYTES = algorithmic bytes per launch)
#   cmd:ARGS         any command (commas become spaces), 300 s limit
# Every GPU step has its own time limit; the script stops at the first failure.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${TAG:-run}
mkdir -p "$O"
cd "$R"
for step in "$@"; do
  kind=${step%%:*}
  arg=${step#*:}; [ "$arg" = "$step" ] && arg=""
  case $kind in
    tests)
      k=(); [ -n "$arg" ] && k=(-k "$arg")
      timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread "${k[@]}" \
        > "$O/gputest.log" 2>&1 || { tail -30 "$O/gputest.log"; exit 1; }
      tail -3 "$O/gputest.log"
      timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
      echo "tests ok" ;;
    bench)
      a=${arg//,/ }; [ -z "$a" ] && a="--steps 20 --warmup 5"
      n=$(ls "$O" | grep -c '^bench' || true)
      timeout -k 10 600 python bench.py $a --detail "$O/bench${n}_detail.json" > "$O/bench$n.json" 2> "$O/bench$n.err" \
        || { tail -20 "$O/bench$n.err"; exit 1; }
      echo "bench$n done: $a" ;;
    prof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$O/prof_$arg" -o run -- python3 "$R/bench.py" --config "$arg" --steps 10 --warmup 2 --timed-only \
        --sub-configs none > "$O/prof_$arg.log" 2>&1) || { tail -20 "$O/prof_$arg.log"; exit 1; }
      echo "profiled $arg" ;;
    pmc)
      IFS=: read -r cfg kern algo <<< "$arg"
      for c in FETCH_SIZE WRITE_SIZE; do
        (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv \
          -d "$O/pmc_${c}_$cfg" -o run -- python3 "$R/bench.py" --config "$cfg" --steps 2 --warmup 1 --serial-calls \
          --timed-only --sub-configs none > "$O/pmc_${c}_$cfg.log" 2>&1) || { tail -20 "$O/pmc_${c}_$cfg.log"; exit 1; }
      done
      python3 "$R/tools/pmc_traffic.py" --fetch "$O/pmc_FETCH_SIZE_$cfg" --write "$O/pmc_WRITE_SIZE_$cfg" \
        --kernel "$kern" --algo-bytes "$algo" --out "$O/pmc_${kern}_$cfg.json"
      echo "pmc $cfg $kern done" ;;
    cmd)
      timeout -k 10 300 ${arg//,/ } ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
