#!/bin/bash
# accumulate jagged pass (K <= 4): next window a whole slice ahead; synth parity + interleaved A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_jag.py "tests/test_gpu_configs.py" \
  > gpurun_out/r03_t13.log 2>&1 || { tail -30 gpurun_out/r03_t13.log; exit 1; }
tail -2 gpurun_out/r03_t13.log
bash tools/ab_env.sh 2 KRCN_LIB $R/scratch/variants/vahead0/libkrcn.so $R/krylov-cubic-regularized-newton_amd/lib/libkrcn.so \
  -- --config synth 2>&1 | tee gpurun_out/r03_ab13.txt
