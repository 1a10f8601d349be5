#!/bin/bash
# w8a A/B (combine rows per block, pass-1 grid; tuning build), then the final evidence (r03_gpu26.sh)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
( export KRCN_LIB=$R/scratch/variants/vtune/libkrcn.so
  bash tools/ab_multi.sh 2 "KRCN_XT_SMALL=0" "KRCN_XT_RB=16" "KRCN_XT_RB=32" "KRCN_XT_RB=64" "KRCN_WIN_ACC_B=128" "KRCN_WIN_ACC_B=128 KRCN_XT_RB=16" -- --config w8a 2>&1 | tee gpurun_out/r03_ab27_w8a_xt.txt ) || exit 1
bash tools/r03_gpu26.sh
