#!/bin/bash
# single-window long rows summed by whole waves: parity, news20 uniform + skewed bench
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_jag.py tests/test_gpu_lanczos.py tests/test_gpu_tiling.py "tests/test_gpu_configs.py::test_news20_crn_trajectory" \
  > gpurun_out/r03_t19.log 2>&1 || { tail -40 gpurun_out/r03_t19.log; exit 1; }
tail -2 gpurun_out/r03_t19.log
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-cold > gpurun_out/r03_b19.log 2>&1 || exit 3
python3 tools/ab_line.py "news20" gpurun_out/r03_b19.log
timeout -k 10 300 python3 bench.py --skew --steps 10 --warmup 3 --no-cpu-baseline --no-cold > gpurun_out/r03_b19s.log 2>&1 || exit 4
python3 tools/ab_line.py "news20 skew" gpurun_out/r03_b19s.log
