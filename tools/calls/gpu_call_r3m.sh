# gemm_x3 (ConvT GEMMs) at 4 resident blocks per CU: parity, same-box A/B against 2, kernel trace of the C2 step
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3m_tests.log 2>&1 || { tail -30 gpurun_out/r3m_tests.log; exit 1; }
tail -3 gpurun_out/r3m_tests.log
bash tools/ab_c4.sh "CDM_GEMM_MINB=2" "CDM_GEMM_MINB=4" 2 | tee gpurun_out/r3m_ab.txt
bash tools/train_step_profile.sh gpurun_out/r3m_prof --math h3 && grep -n "gemm_x3\|kernel sum" gpurun_out/r3m_prof/breakdown.txt
echo ALL_DONE
