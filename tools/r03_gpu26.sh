#!/bin/bash
# round-3 final evidence at HEAD (r03f): full GPU suite + smoke, then bench lines and
# rocprofv3 summaries (kernel stats, FETCH_SIZE, WRITE_SIZE) for all five configs,
# then five fresh news20 processes
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r03f_gpu_full.log 2>&1; rc=$?
tail -3 gpurun_out/r03f_gpu_full.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03f_smoke.log 2>&1 || { tail -5 gpurun_out/r03f_smoke.log; exit 1; }
tail -1 gpurun_out/r03f_smoke.log
bash tools/r03_prof_all.sh r03f w8a rcv1 news20 rcv1_stress synth || exit 1
bash tools/news20_procs.sh 5 r03f_np 2>&1 | tee gpurun_out/r03f_news20_procs.txt
