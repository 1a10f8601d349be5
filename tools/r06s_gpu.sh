# round 6: skewed shapes at HEAD beside the uniform lines, with rocprofv3 summaries
set -o pipefail
bash tools/gpu.sh "bench:r06u:news20:--no-cpu-baseline" "bench:r06u:rcv1:--no-cpu-baseline" \
  "bench:r06s:news20:--skew,--no-cpu-baseline" "bench:r06s:rcv1:--skew,--no-cpu-baseline" || exit 1
bash tools/prof_bench.sh r06s_news20skew --config news20 --skew || exit 1
bash tools/prof_bench.sh r06s_rcv1skew --config rcv1 --skew || exit 1
