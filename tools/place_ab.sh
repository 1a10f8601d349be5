#!/bin/bash
# Interleaved fresh-process A/B of the placement probe (krcn_csr_set_placement_trials):
#   bash tools/place_ab.sh <tag> <reps> [<config>] [<trials values...>]
# each rep runs one fresh bench.py process per trials value (default: 0 = off, -1 = auto).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
tag=$1; reps=$2; cfg=${3:-news20}; shift 3 2>/dev/null
vals=("$@"); [ ${#vals[@]} -eq 0 ] && vals=(0 -1)
for i in $(seq 1 $reps); do
  for v in "${vals[@]}"; do
    timeout -k 10 240 python3 bench.py --config $cfg --no-cpu-baseline --no-cold --steps 10 --placement-trials $v \
      > gpurun_out/${tag}_t${v}_p$i.log 2>&1 || { tail -5 gpurun_out/${tag}_t${v}_p$i.log; exit 1; }
    python3 tools/ab_line.py "trials $v proc $i" gpurun_out/${tag}_t${v}_p$i.log
  done
done 2>&1 | tee gpurun_out/${tag}.txt
