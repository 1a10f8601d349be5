#!/bin/bash
# CGS2 iteration on the GPU box: reorth parity tests, a rcv1_stress bench line
# and a kernel trace summarised per k.  bash tools/cgs_iter.sh <tag>
set -o pipefail
TAG=${1:-x}
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_lanczos.py tests/test_gpu_configs.py > gpurun_out/cgs_test_$TAG.log 2>&1 || { tail -30 gpurun_out/cgs_test_$TAG.log; exit 1; }
tail -1 gpurun_out/cgs_test_$TAG.log
timeout -k 10 200 python bench.py --config rcv1_stress --no-cold --steps 5 --warmup 2 > gpurun_out/cgs_bench_$TAG.log 2>&1 || exit 2
python3 tools/bench_summary.py gpurun_out/cgs_bench_$TAG.log
bash tools/trace_bench.sh $TAG --config rcv1_stress --steps 2 --warmup 1 || exit 3
python3 tools/cgs_trace.py gpurun_out/trace_$TAG/t_kernel_trace.csv
