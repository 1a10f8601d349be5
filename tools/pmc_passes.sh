#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) over a short bench run.
# usage: bash tools/pmc_passes.sh <tag> [bench args...]  -> gpurun_out/pmc_<tag>/<pass>/
set -o pipefail
TAG=${1:-x}; shift
R=$GRAFT_REPO_ROOT
[ -n "$R" ] || R=$(pwd)
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-cold $*"
run() {
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o p -- python3 $R/bench.py $ARGS > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; return $rc
}
run sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD || exit 1
run tcc TCC_HIT_sum TCC_MISS_sum || exit 1
run fetch FETCH_SIZE || exit 1
run ta TA_BUSY_avr TA_BUSY_max || exit 1
python3 $R/tools/pmc_table.py $OUT/sq $OUT/tcc $OUT/fetch $OUT/ta > $OUT/table.txt 2>&1
