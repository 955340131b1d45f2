R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/lik_debug.py > gpurun_out/lik_debug.log 2>&1; cat gpurun_out/lik_debug.log | grep -v amdgpu.ids
timeout -k 10 300 python -u -m pytest tests/test_gpu_likelihood.py -x -q --timeout 200 --timeout-method thread 2>&1 | tail -3
