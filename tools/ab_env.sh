#!/bin/bash
# Interleaved A/B of one environment knob on the GPU box:
#   bash tools/ab_env.sh <reps> <VAR> <value> <value> ... [-- bench args]
# prints HVP/s, the pass-1 plan and the per-launch times of bench.py per run.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
reps=$1; var=$2; shift 2
vals=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do vals+=("$1"); shift; done
[ "$1" == "--" ] && shift
for i in $(seq 1 $reps); do
  for v in "${vals[@]}"; do
    env "$var=$v" timeout -k 10 180 python3 $R/bench.py --steps 10 --warmup 5 --no-cpu-baseline --no-cold "$@" > /tmp/ab_env.log 2>&1 || { echo "FAIL $var=$v"; tail -5 /tmp/ab_env.log; exit 1; }
    python3 $R/tools/ab_line.py "$var=$v" /tmp/ab_env.log
  done
done
