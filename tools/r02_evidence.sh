# Round evidence on the GPU box: bash tools/r02_evidence.sh [tag]   (default r02)
set -o pipefail
T=${1:-r02}
mkdir -p gpurun_out
bash tools/prof_bench.sh $T || exit 1
bash tools/prof_bench.sh ${T}_synth --config synth || exit 1
for c in news20 rcv1 w8a rcv1_stress synth; do
  timeout -k 10 400 python bench.py --config $c > gpurun_out/${T}_bench_$c.json.log 2>&1 || exit 2
  echo "bench $c done"
done
