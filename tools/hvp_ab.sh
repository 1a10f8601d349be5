#!/bin/bash
# interleaved standalone-HVP A/B: old lib vs new lib, news20 bench lines, warm HVP us
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for i in 1 2 3; do
  for lib in scratch/variants/vold/libkrcn.so krylov-cubic-regularized-newton_amd/lib/libkrcn.so; do
    KRCN_LIB=$R/$lib timeout -k 10 200 python3 bench.py --steps 10 --warmup 4 --no-cpu-baseline > /tmp/hab.log 2>&1 || { echo "FAIL $lib"; tail -5 /tmp/hab.log; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open('/tmp/hab.log').read().strip().splitlines()[-1])
print('$lib'.split('/')[-2], round(d['value']), 'warm HVP us', round(d['hvp_warm_us']['median'],2), 'p10', round(d['hvp_warm_us']['p10'],2), 'frac', round(d['hvp_warm_frac']['of_8.0_TBps'],3), 'cold', round(d['hvp_cold_us'],1))" | tee -a gpurun_out/r04_hvp_l2_ab.txt
  done
done
