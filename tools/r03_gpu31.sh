#!/bin/bash
# repeat run 30's sequence with a 120 s per-test timeout: pytest-timeout dumps every thread's stack
# if test_synth_rows_x8_crn_step stalls again (run 30 went silent there for 180 s)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_jag.py tests/test_gpu_window.py tests/test_gpu_tiling.py tests/test_gpu_virtual_shards.py \
  > gpurun_out/r03_t31.log 2>&1; rc=$?
tail -3 gpurun_out/r03_t31.log
exit $rc
