#!/bin/bash
# w8a: rows per tile of the one-piece fused pass (KRCN_WIN_R; the rule picks 16 at 11.6 nonzeros a row), tuning build
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export KRCN_LIB=$R/scratch/variants/vtune/libkrcn.so
bash tools/ab_multi.sh 3 "KRCN_WIN_R=16" "KRCN_WIN_R=32" "KRCN_WIN_R=64" -- --config w8a 2>&1 | tee gpurun_out/r03_ab33_w8a_winr.txt
