#!/bin/bash
# Timing-only ablations of the window pass (run on the GPU box from the repo root):
# bench.py once per library in scratch/variants/v*/ (plus the default), pass times only.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for lib in $R/krylov-cubic-regularized-newton_amd/lib/libkrcn.so $R/krylov-cubic-regularized-newton_amd/../scratch/variants/v*/libkrcn.so; do
  KRCN_LIB=$lib timeout -k 10 120 python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-cold > /tmp/abl.log 2>&1 || { echo "FAIL $lib"; tail -5 /tmp/abl.log; exit 1; }
  python3 -c "
import json,sys;d=json.loads(open('/tmp/abl.log').read().strip().splitlines()[-1]);r=d['roofline']
print(sys.argv[1].split('lib/')[-1], round(d['value']), round(r['pass1_us'],2), round(r['pass2_us'],2))" $lib
done
