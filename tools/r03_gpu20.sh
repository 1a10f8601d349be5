#!/bin/bash
# skewed news20 shape: window tile rows R (tuning build, KRCN_WIN_R)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export KRCN_LIB=$R/scratch/variants/vtune/libkrcn.so
bash tools/ab_env.sh 2 KRCN_WIN_R 16 32 64 -- --skew 2>&1 | tee gpurun_out/r03_ab20.txt
