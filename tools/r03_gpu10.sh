#!/bin/bash
# fused pass 1 prologue / ring rework: news20 parity, then interleaved A/B
# against the round-3 baseline build (scratch/variants/vbase)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_lanczos.py tests/test_gpu_graph.py "tests/test_gpu_configs.py::test_news20_crn_trajectory" \
  > gpurun_out/r03_t10.log 2>&1 || { tail -30 gpurun_out/r03_t10.log; exit 1; }
tail -3 gpurun_out/r03_t10.log
bash tools/ab_env.sh 3 KRCN_LIB $R/scratch/variants/vbase/libkrcn.so $R/krylov-cubic-regularized-newton_amd/lib/libkrcn.so \
  2>&1 | tee gpurun_out/r03_ab10.txt
