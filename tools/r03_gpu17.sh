#!/bin/bash
# synth rank-of-8 rehearsal: pass-2 slice groups at HEAD (tuning build)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export KRCN_LIB=$R/scratch/variants/vtune/libkrcn.so
bash tools/ab_env.sh 2 KRCN_JAG_G 0,1 0,2 0,4 -- --config synth --rehearse-shard 8 2>&1 | tee gpurun_out/r03_ab17.txt
