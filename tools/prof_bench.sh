#!/bin/bash
# rocprofv3 evidence for the bench command (run on the GPU box from the repo root):
#   kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in separate --pmc passes,
#   then the FETCH_SIZE width calibration (tools/fetch_calib.hip).
# usage: bash tools/prof_bench.sh <tag> [bench args...]   -> gpurun_out/prof_<tag>/
set -o pipefail
TAG=${1:-r01}; shift
R=$GRAFT_REPO_ROOT
[ -n "$R" ] || R=$(pwd)
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cp $R/.rev $OUT/rev.txt 2>/dev/null || echo unknown > $OUT/rev.txt
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 5 --warmup 1 --no-cpu-baseline --no-cold $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- python3 $R/bench.py $ARGS > $OUT/trace.log 2>&1; rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o bench -- python3 $R/bench.py $ARGS > $OUT/fetch.log 2>&1; rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o bench -- python3 $R/bench.py $ARGS > $OUT/write.log 2>&1; rc=$?; echo "write rc=$rc"; [ $rc -eq 0 ] || exit $rc
if [ -x $R/tools/fetch_calib ]; then
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/calib -o calib -- $R/tools/fetch_calib > $OUT/calib.log 2>&1; echo "calib rc=$?"
fi
grep -h '"metric"' $OUT/trace.log | head -1
