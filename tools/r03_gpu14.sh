#!/bin/bash
# synth pass 2 slice groups re-measured at HEAD (tuning build): KRCN_JAG_G=0,g
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export KRCN_LIB=$R/scratch/variants/vtune/libkrcn.so
bash tools/ab_env.sh 2 KRCN_JAG_G 0,1 0,2 0,4 -- --config synth 2>&1 | tee gpurun_out/r03_ab14.txt
