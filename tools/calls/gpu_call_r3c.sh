# round-3: BN-backward sums in the dgrad epilogue — kernel + model / trainer / C2 / C4 parity, then the A/B
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_trainer.py tests/test_gpu_c2_e2e.py tests/test_gpu_configs.py tests/test_gpu_rccl.py -x -q --timeout 200 --timeout-method thread > gpurun_out/c5_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/c5_tests.log; exit 1; }
tail -2 gpurun_out/c5_tests.log
bash tools/ab_c4.sh "CDM_BN_SUMS_EPI=0" "CDM_BN_SUMS_EPI=1" 2 > gpurun_out/c5_ab_sums_epi.txt 2>&1 || exit 1
cat gpurun_out/c5_ab_sums_epi.txt
echo ALL_DONE
