#!/bin/bash
# window consume: long-row lanes batch their slab reads (ballot-guarded), lib vs vsu1 (before); uniform + skewed
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_window.py tests/test_gpu_lanczos.py tests/test_gpu_tiling.py \
  > gpurun_out/r03_t22.log 2>&1 || { tail -30 gpurun_out/r03_t22.log; exit 1; }
tail -2 gpurun_out/r03_t22.log
L=$R/krylov-cubic-regularized-newton_amd/lib/libkrcn.so
bash tools/ab_env.sh 3 KRCN_LIB $R/scratch/variants/vsu1/libkrcn.so $L 2>&1 | tee gpurun_out/r03_ab22.txt
bash tools/ab_env.sh 2 KRCN_LIB $R/scratch/variants/vsu1/libkrcn.so $L -- --skew 2>&1 | tee -a gpurun_out/r03_ab22.txt
