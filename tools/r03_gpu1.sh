#!/bin/bash
# round 3, first GPU call: the new virtual-shard parity tests + ADVICE fixes,
# then news20 rows-per-tile A/B on the tuning build.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
  tests/test_gpu_virtual_shards.py tests/test_gpu_graph.py \
  "tests/test_gpu_methods.py::test_sscn_without_stored_products" \
  "tests/test_gpu_methods.py::test_smoothness_mixed_sign_columns" \
  "tests/test_gpu_methods.py::test_cubic_ls_cg_fp32_terminates" \
  "tests/test_gpu_methods.py::test_smoothness_and_hessian_lipschitz" > gpurun_out/r03_t1.log 2>&1
rc=$?
tail -15 gpurun_out/r03_t1.log
KRCN_LIB=$GRAFT_REPO_ROOT/scratch/variants/vtune/libkrcn.so timeout -k 10 400 bash tools/ab_env.sh 2 KRCN_WIN_R 32 64 > gpurun_out/r03_winR.log 2>&1
cat gpurun_out/r03_winR.log
exit $rc
