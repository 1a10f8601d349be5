#!/bin/bash
# Interleaved A/B of environment settings on the GPU box:
#   bash tools/ab_multi.sh <reps> "A=1 B=2" "A=3" ... [-- bench args]
# each setting is a space-separated list of VAR=value; prints one ab_line per run.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
reps=$1; shift
sets=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do sets+=("$1"); shift; done
[ "$1" == "--" ] && shift
for i in $(seq 1 $reps); do
  for st in "${sets[@]}"; do
    env $st timeout -k 10 180 python3 $R/bench.py --steps 10 --warmup 5 --no-cpu-baseline --no-cold "$@" > /tmp/ab_multi.log 2>&1 || { echo "FAIL $st"; tail -5 /tmp/ab_multi.log; exit 1; }
    python3 $R/tools/ab_line.py "$st" /tmp/ab_multi.log
  done
done
