#!/bin/bash
# full GPU suite + smoke at HEAD, the news20 bench line, then synth pass-1 slice groups A/B (tuning build)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r03_gpu_full23.log 2>&1; rc=$?
tail -5 gpurun_out/r03_gpu_full23.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -3 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/r03_bench23_news20.log 2>&1 || { tail -5 gpurun_out/r03_bench23_news20.log; exit 1; }
python tools/ab_line.py news20 gpurun_out/r03_bench23_news20.log
export KRCN_LIB=$R/scratch/variants/vtune/libkrcn.so
bash tools/ab_env.sh 2 KRCN_JAG_G 0,0 2,0 4,0 -- --config synth 2>&1 | tee gpurun_out/r03_ab23_synth_g1.txt
# rcv1: single-window jagged pass 2 (X^T u gathers all of u) with fewer row groups than waves
KRCN_JAG_S1G=256 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_configs.py -k rcv1 > gpurun_out/r03_t23_rcv1_jag.log 2>&1; tail -2 gpurun_out/r03_t23_rcv1_jag.log
bash tools/ab_multi.sh 2 "KRCN_JAG_S1G=4096" "KRCN_JAG_S1G=256" "KRCN_JAG_S1G=256 KRCN_JAG_R=128" "KRCN_JAG_S1G=256 KRCN_JAG_R=64" -- --config rcv1 2>&1 | tee gpurun_out/r03_ab23_rcv1_jag.txt
