set -o pipefail
mkdir -p gpurun_out
bash tools/prof_bench.sh r02 || exit 1
bash tools/prof_bench.sh r02_synth --config synth || exit 1
for c in news20 rcv1 w8a rcv1_stress synth; do
  timeout -k 10 400 python bench.py --config $c > gpurun_out/r02_bench_$c.json.log 2>&1 || exit 2
  echo "bench $c done"
done
