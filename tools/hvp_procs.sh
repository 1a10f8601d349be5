#!/bin/bash
# n fresh news20 bench processes: the Lanczos HVP/s and the standalone warm HVP of each
# (the placement spread).  bash tools/hvp_procs.sh <tag> <n>
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
TAG=${1:-x}; N=${2:-5}
for i in $(seq 1 $N); do
  timeout -k 10 200 python3 bench.py --steps 10 --warmup 4 --no-cpu-baseline > /tmp/hp.log 2>&1 || { echo "FAIL"; tail -5 /tmp/hp.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('/tmp/hp.log').read().strip().splitlines()[-1])
print('proc $i', round(d['value']), 'HVP/s in Lanczos; warm HVP', round(d['hvp_warm_us']['median'],2), 'us =', round(d['hvp_warm_frac']['of_8.0_TBps'],3), 'of 8 TB/s; cold', round(d['hvp_cold_us'],1), 'us')" | tee -a gpurun_out/${TAG}_hvp_procs.txt
done
