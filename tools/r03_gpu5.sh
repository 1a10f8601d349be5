#!/bin/bash
# round 3, GPU call 5: wave-block rounds in the accumulate jagged pass (synth,
# sharded ranks): parity, then synth timing.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread \
  tests/test_gpu_jag.py tests/test_gpu_sharded_paths.py tests/test_gpu_configs.py::test_synth_config \
  tests/test_gpu_virtual_shards.py tests/test_gpu_hvp.py > gpurun_out/r03_t5.log 2>&1
rc=$?
tail -5 gpurun_out/r03_t5.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python3 bench.py --config synth --steps 5 --warmup 2 --no-cpu-baseline --no-cold > /tmp/s.log 2>&1 && python3 tools/ab_line.py "synth waveblock" /tmp/s.log
done
timeout -k 10 300 python3 bench.py --config synth --rehearse-shard 8 --steps 5 --warmup 2 --no-cpu-baseline --no-cold > /tmp/s8.log 2>&1 && python3 tools/ab_line.py "synth rank-of-8" /tmp/s8.log
