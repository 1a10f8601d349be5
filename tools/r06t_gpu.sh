# round 6: skewed-shape fixes (jag long-task capacity; long rows only past 255 when the window is nearly full)
set -o pipefail
bash tools/gpu.sh "suite:r06t2:tests/test_gpu_jag.py,tests/test_gpu_window.py" || exit 1
bash tools/gpu.sh "bench:r06t2:rcv1:--no-cpu-baseline" "bench:r06ts2:rcv1:--skew,--no-cpu-baseline" "bench:r06t2:news20:--no-cpu-baseline" "bench:r06ts2:news20:--skew,--no-cpu-baseline" || exit 1
bash tools/gpu.sh "ab:r06u_coop_ab:2:krylov-cubic-regularized-newton_amd/lib/libkrcn.so:abvar/vcoop/libkrcn.so:--config,news20,--skew" || exit 1
bash tools/gpu.sh "py:r06v_skew_formats_rcv1:tools/skew_formats.py:--config,rcv1,--skew" || exit 1
bash tools/gpu.sh "py:r06v_skew_formats_news20:tools/skew_formats.py:--config,news20,--skew,--p1,0,--p2,0" || exit 1
bash tools/ab_multi.sh 2 "KRCN_LIB=$GRAFT_REPO_ROOT/abvar/vtune/libkrcn.so KRCN_JAG_G=0,1" "KRCN_LIB=$GRAFT_REPO_ROOT/abvar/vtune/libkrcn.so KRCN_JAG_G=0,2" -- --config synth --rehearse-shard 8 2>&1 | tee gpurun_out/r06w_synth8_pass2_groups.txt
