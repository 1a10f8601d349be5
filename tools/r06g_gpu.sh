set -o pipefail
bash tools/gpu.sh "ab:r06e_cgs2_release_ab:2:abvar/vprefence/libkrcn.so:krylov-cubic-regularized-newton_amd/lib/libkrcn.so:--config,rcv1_stress" "suite:r06e:tests/test_gpu_lanczos.py,-k,reorth" || exit 1
KRCN_LIB=$GRAFT_REPO_ROOT/abvar/vfold/libkrcn.so timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_lanczos.py -k "early_alpha or news20_shape or deterministic" > gpurun_out/r06g_fold_tests.log 2>&1 || { tail -30 gpurun_out/r06g_fold_tests.log; exit 1; }
tail -2 gpurun_out/r06g_fold_tests.log
bash tools/gpu.sh "ab:r06g_fold_ab:3:krylov-cubic-regularized-newton_amd/lib/libkrcn.so:abvar/vfold/libkrcn.so:--config,news20" || exit 1
bash tools/ab.sh 2 krylov-cubic-regularized-newton_amd/lib/libkrcn.so abvar/vpst2/libkrcn.so abvar/vvst2/libkrcn.so -- --config news20 2>&1 | tee gpurun_out/r06g_nt_stores_ab.txt
