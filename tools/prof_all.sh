#!/bin/bash
# rocprof evidence + full bench lines for a list of configs (run on the GPU box):
#   bash tools/prof_all.sh <tag> <cfg> [<cfg> ...]
#   -> gpurun_out/prof_<tag>_<cfg>/ (trace, fetch, write) and gpurun_out/<tag>_bench_<cfg>.json
set -o pipefail
R=$GRAFT_REPO_ROOT
[ -n "$R" ] || R=$(pwd)
TAG=$1; shift
mkdir -p $R/gpurun_out
for cfg in "$@"; do
  steps=20; [ "$cfg" = synth ] && steps=10; [ "$cfg" = rcv1_stress ] && steps=5
  (cd $R && timeout -k 10 400 python3 bench.py --config $cfg --steps $steps --warmup 3 > gpurun_out/${TAG}_bench_$cfg.log 2>&1) || { echo "bench $cfg failed"; tail -5 $R/gpurun_out/${TAG}_bench_$cfg.log; exit 1; }
  grep '"metric"' $R/gpurun_out/${TAG}_bench_$cfg.log > $R/gpurun_out/${TAG}_bench_$cfg.json
  python3 $R/tools/ab_line.py "$cfg" $R/gpurun_out/${TAG}_bench_$cfg.json
  bash $R/tools/prof_bench.sh ${TAG}_$cfg --config $cfg || exit 1
done
