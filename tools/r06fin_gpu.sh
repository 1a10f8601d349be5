# round 6 final evidence at the committed tree (.rev), in two calls:
#   bash tools/r06fin_gpu.sh a   full -m gpu suite, smoke, news20 / rcv1 / w8a lines + rocprofv3
#   bash tools/r06fin_gpu.sh b   rcv1_stress / synth lines + rocprofv3, rank-of-8 rehearsals,
#                                skewed lines + rocprofv3, five fresh news20 processes
set -o pipefail
case "$1" in
  a)
    bash tools/gpu.sh suite:r06fin_suite smoke:r06fin || exit 1
    bash tools/prof_all.sh r06fin news20 rcv1 w8a || exit 1 ;;
  b)
    bash tools/prof_all.sh r06fin rcv1_stress synth || exit 1
    bash tools/gpu.sh "profr:r06fin:news20:8" "profr:r06fin:synth:8" || exit 1
    bash tools/gpu.sh "bench:r06fins:rcv1:--skew" "bench:r06fins:news20:--skew" || exit 1
    bash tools/prof_bench.sh r06fin_rcv1skew --config rcv1 --skew || exit 1
    bash tools/prof_bench.sh r06fin_news20skew --config news20 --skew || exit 1
    bash tools/gpu.sh "procs:r06fin_news20:5" || exit 1 ;;
esac
