#!/bin/bash
# slice-group cost model refit: synth pass 2 at G = 2; parity + bench + rank rehearsals
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_jag.py tests/test_gpu_configs.py tests/test_gpu_virtual_shards.py tests/test_gpu_lanczos.py tests/test_gpu_sharded_paths.py \
  > gpurun_out/r03_t15.log 2>&1 || { tail -30 gpurun_out/r03_t15.log; exit 1; }
tail -2 gpurun_out/r03_t15.log
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --config synth --steps 10 --warmup 3 --no-cold > gpurun_out/r03_b15_synth_$i.log 2>&1 || exit 3
  python3 tools/ab_line.py "synth 1-GPU run $i" gpurun_out/r03_b15_synth_$i.log
done
for N in 2 4 8; do
  timeout -k 10 300 python3 bench.py --config synth --rehearse-shard $N --steps 10 --warmup 3 --no-cpu-baseline --no-cold > gpurun_out/r03_b15_reh$N.log 2>&1 || exit 4
  python3 tools/ab_line.py "synth rank-of-$N" gpurun_out/r03_b15_reh$N.log
done
