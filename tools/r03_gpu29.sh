#!/bin/bash
# HEAD (chunked per-block X^T copies): full GPU suite + smoke, then the w8a bench line and rocprofv3 summary (r03g)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r03g_gpu_full.log 2>&1; rc=$?
tail -3 gpurun_out/r03g_gpu_full.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03g_smoke.log 2>&1 || { tail -5 gpurun_out/r03g_smoke.log; exit 1; }
tail -1 gpurun_out/r03g_smoke.log
bash tools/r03_prof_all.sh r03g w8a news20 || exit 1
