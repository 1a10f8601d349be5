#!/bin/bash
# chunked per-block X^T copies (w8a): parity, then fused vs separate X^T pass on uniform and skewed w8a shapes
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_window.py tests/test_gpu_lanczos.py tests/test_gpu_configs.py tests/test_gpu_graph.py tests/test_gpu_crn.py \
  > gpurun_out/r03_t28.log 2>&1 || { tail -30 gpurun_out/r03_t28.log; exit 1; }
tail -2 gpurun_out/r03_t28.log
export KRCN_LIB=$R/scratch/variants/vtune/libkrcn.so
bash tools/ab_multi.sh 3 "KRCN_XT_SMALL=0" "KRCN_XT_SMALL=1" -- --config w8a 2>&1 | tee gpurun_out/r03_ab28_w8a_xt.txt
bash tools/ab_multi.sh 2 "KRCN_XT_SMALL=0" "KRCN_XT_SMALL=1" -- --config w8a --skew 2>&1 | tee gpurun_out/r03_ab28_w8a_skew_xt.txt
