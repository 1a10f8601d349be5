#!/bin/bash
# single-window jagged pass: first chunk issued with the window fetch; parity + news20 A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_jag.py tests/test_gpu_lanczos.py "tests/test_gpu_configs.py::test_news20_crn_trajectory" tests/test_gpu_graph.py \
  > gpurun_out/r03_t16.log 2>&1 || { tail -30 gpurun_out/r03_t16.log; exit 1; }
tail -2 gpurun_out/r03_t16.log
bash tools/ab_env.sh 3 KRCN_LIB $R/scratch/variants/vje0/libkrcn.so $R/krylov-cubic-regularized-newton_amd/lib/libkrcn.so \
  2>&1 | tee gpurun_out/r03_ab16.txt
