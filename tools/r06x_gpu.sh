# round 6: after the skew / rank pass-2 changes: the affected GPU suites, then the lines
set -o pipefail
bash tools/gpu.sh "suite:r06x:tests/test_gpu_jag.py,tests/test_gpu_window.py,tests/test_gpu_virtual_shards.py,tests/test_gpu_lanczos.py" || exit 1
bash tools/gpu.sh "bench:r06x:rcv1:--no-cpu-baseline" "bench:r06xs:rcv1:--skew,--no-cpu-baseline" "bench:r06xs:news20:--skew,--no-cpu-baseline" "bench:r06x:news20:--no-cpu-baseline" || exit 1
bash tools/gpu.sh "profr:r06x:synth:8" || exit 1
