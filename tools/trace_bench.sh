#!/bin/bash
# Kernel trace + stats of a short bench run: bash tools/trace_bench.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-x}; shift
R=$GRAFT_REPO_ROOT
[ -n "$R" ] || R=$(pwd)
OUT=$R/gpurun_out/trace_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o t -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-cold "$@" > $OUT/run.log 2>&1
rc=$?; echo "trace $TAG rc=$rc"; exit $rc
