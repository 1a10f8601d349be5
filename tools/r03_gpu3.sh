#!/bin/bash
# round 3, third GPU call: pair-level jagged pass + removed w probe:
# the GPU parity tests that cover jagged plans, then news20 A/B against the
# previous (level-order) tuning build.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_trace_batch.py tests/test_libsvm.py > gpurun_out/r03_t3.log 2>&1
rc=$?
tail -25 gpurun_out/r03_t3.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  KRCN_W_PROBE=0 KRCN_LIB=$R/scratch/variants/vtune/libkrcn.so timeout -k 10 200 python3 bench.py --steps 10 --warmup 5 --no-cpu-baseline --no-cold > /tmp/a.log 2>&1 && python3 tools/ab_line.py "level-order(vtune)" /tmp/a.log
  timeout -k 10 200 python3 bench.py --steps 10 --warmup 5 --no-cpu-baseline --no-cold > /tmp/b.log 2>&1 && python3 tools/ab_line.py "pair-level(HEAD)" /tmp/b.log
done | tee gpurun_out/r03_pairs_ab.log
timeout -k 10 300 python3 bench.py --config synth --steps 5 --warmup 2 --no-cpu-baseline --no-cold > /tmp/s.log 2>&1 && python3 tools/ab_line.py "synth HEAD" /tmp/s.log
