#!/bin/bash
# window consume: slab reads batched per lane (lib: 4, vsu8: 8, vsu1: 1 = before); parity + uniform/skewed A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_window.py tests/test_gpu_lanczos.py "tests/test_gpu_configs.py::test_news20_crn_trajectory" \
  > gpurun_out/r03_t21.log 2>&1 || { tail -30 gpurun_out/r03_t21.log; exit 1; }
tail -2 gpurun_out/r03_t21.log
L=$R/krylov-cubic-regularized-newton_amd/lib/libkrcn.so
bash tools/ab_env.sh 2 KRCN_LIB $R/scratch/variants/vsu1/libkrcn.so $L $R/scratch/variants/vsu8/libkrcn.so 2>&1 | tee gpurun_out/r03_ab21.txt
bash tools/ab_env.sh 1 KRCN_LIB $R/scratch/variants/vsu1/libkrcn.so $L $R/scratch/variants/vsu8/libkrcn.so -- --skew 2>&1 | tee -a gpurun_out/r03_ab21.txt
