#!/bin/bash
# the new plan test (rcv1 jagged X^T, fp64 only) + the jagged and window suites at HEAD
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_jag.py tests/test_gpu_window.py tests/test_gpu_tiling.py tests/test_gpu_virtual_shards.py \
  > gpurun_out/r03_t30.log 2>&1; rc=$?
tail -3 gpurun_out/r03_t30.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r03_t30.log | head; exit $rc; }
