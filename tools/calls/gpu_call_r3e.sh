# round-3: interleaved two-deep weight-gradient staging — bit-exactness vs one-ahead, then the A/B
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread -k "deep_staging or bn_bwd_fused or producer_bn_sums or wgrad" > gpurun_out/c7_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/c7_tests.log; exit 1; }
tail -2 gpurun_out/c7_tests.log
bash tools/ab_c4.sh "CDM_WGRAD_DEEP=0" "CDM_WGRAD_DEEP=1" 2 > gpurun_out/c7_ab.txt 2>&1 || exit 1
cat gpurun_out/c7_ab.txt
echo ALL_DONE
