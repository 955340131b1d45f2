# ConvT GEMMs in the operand-sharing block order: kernel + model parity, then same-box A/B of the train steps and a
# kernel trace of the C2 step under the new order
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3l_tests.log 2>&1 || { tail -30 gpurun_out/r3l_tests.log; exit 1; }
tail -3 gpurun_out/r3l_tests.log
bash tools/ab_c4.sh "CDM_GEMM_ORDER=0" "CDM_GEMM_ORDER=1" 2 | tee gpurun_out/r3l_ab.txt
bash tools/train_step_profile.sh gpurun_out/r3l_prof --math h3 && head -20 gpurun_out/r3l_prof/breakdown.txt
echo ALL_DONE
