#!/bin/bash
# N news20 bench processes in a row (placement spread): pass times and the
# w / partials probe's pick.  bash tools/news20_procs.sh <N> [tag]
N=${1:-6}; TAG=${2:-pp}
for i in $(seq 1 $N); do
  KRCN_W_PROBE_LOG=1 timeout -k 10 150 python bench.py --no-cpu-baseline --no-cold --steps 10 > gpurun_out/${TAG}_$i.log 2>&1 || exit 3
  python3 - gpurun_out/${TAG}_$i.log $i <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if "w probe" in l:
        print("  ", l.strip())
    if l.startswith('{"metric"'):
        d = json.loads(l); L = d["roofline"]["launches"]
        print("run", sys.argv[2], round(d["value"]), "p1", L["pass1"]["avg_us"], "c", L["combine"]["avg_us"], "p2", L["pass2"]["avg_us"])
PY
done
