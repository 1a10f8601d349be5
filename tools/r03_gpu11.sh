#!/bin/bash
# round-3 final bench lines for all five configs (traffic from profiles/traffic.json)
# and five fresh news20 processes (placement spread)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for cfg in news20 rcv1 w8a rcv1_stress synth; do
  steps=20; [ "$cfg" = synth ] && steps=10; [ "$cfg" = rcv1_stress ] && steps=5
  timeout -k 10 400 python3 bench.py --config $cfg --steps $steps --warmup 3 > gpurun_out/r03c_bench_$cfg.log 2>&1 \
    || { echo "bench $cfg failed"; tail -5 gpurun_out/r03c_bench_$cfg.log; exit 1; }
  grep '"metric"' gpurun_out/r03c_bench_$cfg.log > gpurun_out/r03c_bench_$cfg.json
  python3 tools/ab_line.py "$cfg" gpurun_out/r03c_bench_$cfg.json
done
for i in 1 2 3 4 5; do
  timeout -k 10 150 python3 bench.py --no-cpu-baseline --no-cold --steps 10 > gpurun_out/r03c_proc_$i.log 2>&1 || exit 3
  python3 tools/ab_line.py "news20 process $i" gpurun_out/r03c_proc_$i.log
done 2>&1 | tee gpurun_out/r03c_news20_procs.txt
