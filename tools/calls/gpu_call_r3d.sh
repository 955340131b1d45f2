# round-3: two-deep staging (bf16 forward halo conv, kernel-row weight gradient) — bit-exactness vs one-ahead,
# precise bf16 conv test, model / trainer / C2 / C4 parity, then the A/B
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_configs.py tests/test_gpu_model.py tests/test_gpu_c2_e2e.py -x -q --timeout 300 --timeout-method thread > gpurun_out/c6_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/c6_tests.log; exit 1; }
tail -2 gpurun_out/c6_tests.log
bash tools/ab_c4.sh "CDM_HALO_DEEP=0 CDM_WGRAD_DEEP=0" "CDM_HALO_DEEP=1 CDM_WGRAD_DEEP=1" 2 > gpurun_out/c6_ab_deep.txt 2>&1 || exit 1
bash tools/ab_c4.sh "CDM_HALO_DEEP=0 CDM_WGRAD_DEEP=1" "CDM_HALO_DEEP=1 CDM_WGRAD_DEEP=0" 1 >> gpurun_out/c6_ab_deep.txt 2>&1 || exit 1
bash tools/ab_c4.sh "CDM_HALO_ONEB_BWD=0" "CDM_HALO_ONEB_BWD=1" 1 >> gpurun_out/c6_ab_deep.txt 2>&1 || exit 1
cat gpurun_out/c6_ab_deep.txt
echo ALL_DONE
