#!/bin/bash
# skewed news20-shaped problem (lognormal rows, power-law columns): formats and throughput
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 300 python3 bench.py --skew --steps 10 --warmup 3 --no-cpu-baseline --no-cold > gpurun_out/r03_skew.log 2>&1 || { tail -20 gpurun_out/r03_skew.log; exit 1; }
python3 tools/ab_line.py "news20 skew" gpurun_out/r03_skew.log
python3 - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/r03_skew.log") if l.startswith('{"metric"')][-1])
print(d["roofline"]["formats"], d["roofline"]["plan"], d["value"])
PY
