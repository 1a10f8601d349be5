#!/bin/bash
# full GPU suite (fused X^T for one-piece plans; jagged X^T for rcv1-sized u), then A/Bs (tuning build)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r03_gpu_full24.log 2>&1; rc=$?
tail -5 gpurun_out/r03_gpu_full24.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|error" gpurun_out/r03_gpu_full24.log | head -20; exit $rc; }
export KRCN_LIB=$R/scratch/variants/vtune/libkrcn.so
bash tools/ab_multi.sh 3 "KRCN_XT_SMALL=0" "KRCN_XT_SMALL=1 KRCN_XT_COMB=0" "KRCN_XT_SMALL=1" -- --config w8a 2>&1 | tee gpurun_out/r03_ab24_w8a_xt.txt
bash tools/ab_multi.sh 3 "KRCN_JAG_S1G=4096" "KRCN_JAG_S1G=0" -- --config rcv1 2>&1 | tee gpurun_out/r03_ab24_rcv1_jag.txt
bash tools/ab_multi.sh 2 "KRCN_JAG_S1G=4096" "KRCN_JAG_S1G=0" -- --config rcv1_stress 2>&1 | tee gpurun_out/r03_ab24_rcv1s_jag.txt
