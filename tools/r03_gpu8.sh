#!/bin/bash
# round 3, GPU call 8: overlapped row-shard pass 2 — parity (bitwise vs serial,
# 1-rank RCCL and 8 virtual ranks), the sharded tests, then the rank-of-8
# rehearsal A/B of the overlap (tuning build).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread \
  tests/test_gpu_virtual_shards.py tests/test_gpu_sharded_paths.py > gpurun_out/r03_t8.log 2>&1
rc=$?
tail -5 gpurun_out/r03_t8.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do for o in 0 1; do
  KRCN_OVERLAP=$o KRCN_LIB=$R/scratch/variants/vtune/libkrcn.so timeout -k 10 300 python3 bench.py --config synth --rehearse-shard 8 --steps 10 --warmup 3 --no-cpu-baseline --no-cold > gpurun_out/r03_reh8_$o.json 2>&1 && python3 tools/ab_line.py "synth rank-of-8 overlap=$o" gpurun_out/r03_reh8_$o.json
done; done
for n in 2 4; do
  timeout -k 10 300 python3 bench.py --config synth --rehearse-shard $n --steps 10 --warmup 3 --no-cpu-baseline --no-cold > gpurun_out/r03_reh$n.json 2>&1 && python3 tools/ab_line.py "synth rank-of-$n" gpurun_out/r03_reh$n.json
done
