#!/bin/bash
# round 3, second GPU call: rocprof evidence at HEAD (64-row tiles) for news20,
# PMC of the jagged passes (news20 pass 2, synth passes), and the w-probe A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
bash tools/prof_bench.sh r03a_news20 || exit 1
bash tools/pmc_passes.sh r03_news20 || exit 1
bash tools/pmc_passes.sh r03_synth --config synth || exit 1
cd $R
KRCN_LIB=$R/scratch/variants/vtune/libkrcn.so timeout -k 10 600 bash tools/ab_env.sh 4 KRCN_W_PROBE 1 0 > gpurun_out/r03_wprobe.log 2>&1
cat gpurun_out/r03_wprobe.log
cat gpurun_out/pmc_r03_news20/table.txt gpurun_out/pmc_r03_synth/table.txt
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_trace_batch.py > gpurun_out/r03_trace_batch.log 2>&1; tail -6 gpurun_out/r03_trace_batch.log
timeout -k 10 200 python tools/loss_iterates_ab.py news20 100 > gpurun_out/r03_loss_iterates.log 2>&1; cat gpurun_out/r03_loss_iterates.log
