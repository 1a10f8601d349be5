#!/bin/bash
# One driver for the GPU-box runs (replaces round 3's tools/r03_gpuN.sh one-offs).
# Run from the repo root on the box:
#   gpurun -- bash tools/gpu.sh <step> [<step> ...]
# Steps run in order and stop at the first failure (a failed, aborted or
# timed-out GPU step ends the call: nothing more touches the GPU).  A step is
# name:arg1:arg2..., logs go to gpurun_out/<tag>*.log:
#   suite:<tag>[:<pytest files/-k ...>]  the -m gpu suite (or the named files)
#   smoke:<tag>                          __graft_entry__.smoke()
#   bench:<tag>:<cfg>[:<bench args>]     one bench.py line -> gpurun_out/<tag>_bench_<cfg>.json
#   prof:<tag>:<cfg>                     bench line + rocprofv3 stats / FETCH / WRITE (tools/prof_bench.sh)
#   profr:<tag>:<cfg>:<N>                the same for the rank-of-N rehearsal (fill_traffic.py --key <cfg>:rehearse<N>)
#   procs:<tag>:<n>[:<cfg>]              n fresh bench processes (placement spread)
#   ab:<tag>:<reps>:<lib A>:<lib B>[:<bench args>]  interleaved A/B of two libkrcn.so builds
#   abtree:<tag>:<reps>:<dir A>:<dir B>[:<bench args>]  interleaved A/B of two trees' bench.py (old worktrees)
#   abenv:<tag>:<reps>:<VAR=x,VAR2=y>...[:--:<bench args>]  interleaved A/B of env settings
#                                        (KRCN_LIB=$GRAFT_REPO_ROOT/abvar/vtune/libkrcn.so for knobs)
#   probe:<tag>:<reps>[:serial][:old]    tools/virtual_stall_probe.py (old: the round-3 tree under scratch/oldhead)
#   py:<tag>:<script>[:args]             any python tool under a 300 s limit
# Commas inside an argument stand for spaces (bench args: --config,rcv1,--steps,20).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
sp() { echo "${1//,/ }"; }

run_step() {
  local a
  IFS=':' read -r -a a <<< "$1"
  local name=${a[0]} tag=${a[1]}
  echo "=== $1 ($(date +%T))"
  case "$name" in
    suite)
      local files=${a[2]:-tests}
      timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu $(sp "$files") \
        > gpurun_out/${tag}.log 2>&1; local rc=$?
      tail -3 gpurun_out/${tag}.log
      [ $rc -eq 0 ] || { grep -E "FAILED|Error|Timeout" gpurun_out/${tag}.log | head -20; return $rc; } ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 \
        || { tail -20 gpurun_out/${tag}_smoke.log; return 1; }
      tail -1 gpurun_out/${tag}_smoke.log ;;
    bench)
      local cfg=${a[2]}
      timeout -k 10 400 python3 bench.py --config $cfg $(sp "${a[3]}") > gpurun_out/${tag}_bench_$cfg.log 2>&1 \
        || { tail -8 gpurun_out/${tag}_bench_$cfg.log; return 1; }
      grep '"metric"' gpurun_out/${tag}_bench_$cfg.log > gpurun_out/${tag}_bench_$cfg.json
      python3 tools/ab_line.py "$cfg" gpurun_out/${tag}_bench_$cfg.json ;;
    prof)
      bash tools/prof_all.sh $tag ${a[2]} || return 1 ;;
    profr)   # profr:<tag>:<cfg>:<N>: rehearsal line (rank 0 of N) + its rocprofv3 stats / FETCH / WRITE
      local cfg=${a[2]} nr=${a[3]}
      local bt=${tag}_rehearse${nr}_$cfg   # (not ${tag}_bench_$cfg: a bench step of the same tag keeps its line)
      timeout -k 10 400 python3 bench.py --config $cfg --rehearse-shard $nr --steps 10 --warmup 3 \
        > gpurun_out/$bt.log 2>&1 || { tail -8 gpurun_out/$bt.log; return 1; }
      grep '"metric"' gpurun_out/$bt.log > gpurun_out/$bt.json
      python3 tools/ab_line.py "$cfg rank of $nr" gpurun_out/$bt.json
      bash tools/prof_bench.sh ${tag}_$cfg$nr --config $cfg --rehearse-shard $nr || return 1 ;;   # (not prof_${tag}_$cfg: a prof step keeps its data)
    procs)
      local n=${a[2]} cfg=${a[3]:-news20}
      for i in $(seq 1 $n); do
        timeout -k 10 200 python3 bench.py --config $cfg --no-cpu-baseline --no-cold --steps 10 \
          > gpurun_out/${tag}_p$i.log 2>&1 || { tail -5 gpurun_out/${tag}_p$i.log; return 1; }
        python3 tools/ab_line.py "proc $i" gpurun_out/${tag}_p$i.log
      done ;;
    ab)
      local reps=${a[2]} la=${a[3]} lb=${a[4]}
      for i in $(seq 1 $reps); do
        for lib in "$la" "$lb"; do
          KRCN_LIB=$R/$lib timeout -k 10 200 python3 bench.py --steps 10 --warmup 5 --no-cpu-baseline --no-cold \
            $(sp "${a[5]}") > /tmp/ab.log 2>&1 || { echo "FAIL $lib"; tail -5 /tmp/ab.log; return 1; }
          python3 tools/ab_line.py "$lib" /tmp/ab.log
        done
      done 2>&1 | tee gpurun_out/${tag}.txt ;;
    abtree)   # abtree:<tag>:<reps>:<dir A>:<dir B>[:<bench args>]: interleaved A/B of two source trees
      local reps=${a[2]} da=${a[3]} db=${a[4]}
      for i in $(seq 1 $reps); do
        for dd in "$da" "$db"; do
          (cd $R/$dd && timeout -k 10 200 python3 bench.py --steps 10 --warmup 5 --no-cpu-baseline --no-cold \
            $(sp "${a[5]}") > /tmp/abt.log 2>&1) || { echo "FAIL $dd"; tail -5 /tmp/abt.log; return 1; }
          python3 tools/ab_line.py "$dd" /tmp/abt.log
        done
      done 2>&1 | tee gpurun_out/${tag}.txt ;;
    abenv)
      local reps=${a[2]} sets=() i=3
      while [ $i -lt ${#a[@]} ] && [ "${a[$i]}" != "--" ]; do sets+=("$(sp "${a[$i]}")"); i=$((i + 1)); done
      local extra=""; [ $i -lt ${#a[@]} ] && extra=$(sp "${a[$((i + 1))]}")
      bash tools/ab_multi.sh $reps "${sets[@]}" -- $extra 2>&1 | tee gpurun_out/${tag}.txt ;;
    probe)
      local reps=${a[2]} ser="" dir=$R
      for x in "${a[@]:3}"; do
        [ "$x" = serial ] && ser=--serial
        [ "$x" = old ] && dir=$R/scratch/oldhead
      done
      timeout -k 10 900 python3 -u $dir/tools/virtual_stall_probe.py --reps $reps $ser \
        > gpurun_out/${tag}_probe.log 2>&1; local rc=$?
      grep -E "^rep|synth problem" gpurun_out/${tag}_probe.log | tail -40
      [ $rc -eq 0 ] || { tail -60 gpurun_out/${tag}_probe.log; return $rc; } ;;
    py)
      timeout -k 10 300 python3 -u ${a[2]} $(sp "${a[3]}") > gpurun_out/${tag}.log 2>&1 \
        || { tail -20 gpurun_out/${tag}.log; return 1; }
      tail -15 gpurun_out/${tag}.log ;;
    *) echo "unknown step $name"; return 2 ;;
  esac
}

for st in "$@"; do
  run_step "$st" || { echo "step '$st' failed: stopping"; exit 1; }
done
