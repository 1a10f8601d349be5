#!/bin/bash
# round 3, GPU call 4: pass 2 re-forms z_j (no z store in the fused pass 1):
# Lanczos / graph / config parity, then news20 A/B of KRCN_ZW on the tuning build.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_lanczos.py tests/test_gpu_graph.py tests/test_gpu_crn.py tests/test_gpu_configs.py \
  tests/test_gpu_window.py tests/test_gpu_virtual_shards.py > gpurun_out/r03_t4.log 2>&1
rc=$?
tail -5 gpurun_out/r03_t4.log
[ $rc -eq 0 ] || exit $rc
KRCN_LIB=$R/scratch/variants/vtune/libkrcn.so timeout -k 10 600 bash tools/ab_env.sh 3 KRCN_ZW 0 1 > gpurun_out/r03_zw_ab.log 2>&1
cat gpurun_out/r03_zw_ab.log
