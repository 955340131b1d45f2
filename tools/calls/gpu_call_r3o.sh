# row forms of the C_in = 1 forward / C_out = 1 input gradient: bit-exact vs the flat kernels, model parity, A/B, trace
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3o_tests.log 2>&1 || { tail -30 gpurun_out/r3o_tests.log; exit 1; }
tail -3 gpurun_out/r3o_tests.log
bash tools/ab_c4.sh "CDM_ROW_KERNELS=0" "CDM_ROW_KERNELS=1" 2 | tee gpurun_out/r3o_ab.txt
bash tools/train_step_profile.sh gpurun_out/r3o_prof --math h3 && grep -n "cin1\|cout1\|stats_mm\|kernel sum" gpurun_out/r3o_prof/breakdown.txt
echo ALL_DONE
