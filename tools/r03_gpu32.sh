#!/bin/bash
# final HEAD: full GPU suite + smoke + the default bench line
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread \
  > gpurun_out/r03h_gpu_full.log 2>&1; rc=$?
tail -3 gpurun_out/r03h_gpu_full.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03h_smoke.log 2>&1 || { tail -5 gpurun_out/r03h_smoke.log; exit 1; }
tail -1 gpurun_out/r03h_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r03h_bench_news20.log 2>&1 || { tail -5 gpurun_out/r03h_bench_news20.log; exit 1; }
python tools/ab_line.py news20 gpurun_out/r03h_bench_news20.log
