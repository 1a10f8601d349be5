#!/bin/bash
# Interleaved A/B of library builds on the GPU box (box-to-box variance is a
# few %, so variants are compared within one call):
#   bash tools/ab.sh <reps> <libA> <libB> ... [-- bench args]   (paths relative to the repo root)
# prints HVP/s and the per-launch times of bench.py for each run.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
reps=$1; shift
libs=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do libs+=("$1"); shift; done
[ "$1" == "--" ] && shift
for i in $(seq 1 $reps); do
  for lib in "${libs[@]}"; do
    KRCN_LIB=$R/$lib timeout -k 10 180 python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-cold "$@" > /tmp/ab.log 2>&1 || { echo "FAIL $lib"; tail -5 /tmp/ab.log; exit 1; }
    python3 -c "
import json,sys;d=json.loads(open('/tmp/ab.log').read().strip().splitlines()[-1]);L=d['roofline']['launches']
print(f\"{sys.argv[1]:60s} {d['value']:8.0f} HVP/s  \" + '  '.join(f\"{k} {v['avg_us']:6.2f}\" for k,v in L.items()))" $lib
  done
done
