R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/c3_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/c3_tests.log; exit 1; }
tail -2 gpurun_out/c3_tests.log
bash tools/ab_c4.sh "CDM_EPI_WIDE=0" "CDM_EPI_WIDE=1" 2 > gpurun_out/c3_ab_wide.txt 2>&1 || exit 1
cat gpurun_out/c3_ab_wide.txt
bash tools/ab_c4.sh "CDM_HALO_ONEB=0" "CDM_HALO_ONEB=1" 1 > gpurun_out/c3_ab_oneb.txt 2>&1 || exit 1
cat gpurun_out/c3_ab_oneb.txt
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/fc -o fc -- $R/tools/fetch_calib > $R/gpurun_out/fc.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/fck -o fck -- $R/tools/fetch_calib >> $R/gpurun_out/fc.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r3_rccl -o rccl -- python3 $R/tools/rccl_trace.py > $R/gpurun_out/rccl.log 2>&1 || exit 1
echo ALL_DONE
