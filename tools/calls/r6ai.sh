# round 6 (ai): the extended cross-process bit-exactness test (round-6 schedule switches vs the previous schedules)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6ai
timeout -k 10 600 python -u -m pytest -v -x --timeout 500 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "deep_staging_bit_exact" > gpurun_out/r6ai/tests.log 2>&1; echo "rc=$?"; tail -15 gpurun_out/r6ai/tests.log
echo ALL_DONE
