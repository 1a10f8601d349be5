#!/bin/bash
# Interleaved A/B of the Lanczos hipGraph replay (KRCN_GRAPH=0 eager vs 1)
# on the GPU box:  bash tools/graph_ab.sh <reps> <config>...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
reps=$1; shift
for i in $(seq 1 $reps); do
  for cfg in "$@"; do
    for gr in 0 1; do
      KRCN_GRAPH=$gr timeout -k 10 240 python3 $R/bench.py --config $cfg --steps 20 --warmup 8 --no-cpu-baseline --no-cold > /tmp/gab.log 2>&1 || { echo "FAIL $cfg graph=$gr"; tail -5 /tmp/gab.log; exit 1; }
      python3 -c "
import json,sys;d=json.loads(open('/tmp/gab.log').read().strip().splitlines()[-1])
print(f\"{sys.argv[1]:12s} graph={sys.argv[2]} {d['value']:9.0f} HVP/s {d['ms_per_step']:8.3f} ms/step\")" $cfg $gr
    done
  done
done
