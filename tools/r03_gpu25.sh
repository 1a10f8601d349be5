#!/bin/bash
# parity for the touched paths, then w8a: combine rows per block and the pass-1 grid (tuning build)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_window.py tests/test_gpu_lanczos.py tests/test_gpu_configs.py tests/test_gpu_jag.py tests/test_gpu_graph.py \
  > gpurun_out/r03_t25.log 2>&1 || { tail -30 gpurun_out/r03_t25.log; exit 1; }
tail -2 gpurun_out/r03_t25.log
export KRCN_LIB=$R/scratch/variants/vtune/libkrcn.so
bash tools/ab_multi.sh 3 "KRCN_XT_SMALL=0" "KRCN_XT_RB=16" "KRCN_XT_RB=32" "KRCN_XT_RB=64" "KRCN_WIN_ACC_B=128" "KRCN_WIN_ACC_B=128 KRCN_XT_RB=16" -- --config w8a 2>&1 | tee gpurun_out/r03_ab25_w8a_xt.txt
