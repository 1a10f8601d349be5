#!/bin/bash
# debug: where does the virtual-rank CRN step stall with the overlapped pass 2?
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 200 python -u -m pytest -x -v --timeout 90 --timeout-method thread \
  "tests/test_gpu_virtual_shards.py::test_synth_rows_x8_crn_step" 2>&1 | tee gpurun_out/r03_t9.log
timeout -k 10 200 python -u -m pytest -x -v --timeout 90 --timeout-method thread \
  "tests/test_gpu_virtual_shards.py::test_synth_rows_overlap_bitwise" 2>&1 | tee gpurun_out/r03_t9b.log
