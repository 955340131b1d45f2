# round 4 (l): host RNG / CPU-oracle T=1500 reproduction on the box; bn-sums test fix; band/embed kernels
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -s tests/test_gpu_sampler.py -k "host_rng or host_schedule" > gpurun_out/r4l_rng.log 2>&1; echo "rng rc=$?"
grep -E "PASS|FAIL|host CPU|schedule entries|assert" gpurun_out/r4l_rng.log | head
timeout -k 10 300 python -u tools/t1500_cpu.py --modes fp32 > gpurun_out/r4l_t1500_cpu.txt 2>&1; echo "cpu loop rc=$?"; cat gpurun_out/r4l_t1500_cpu.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_model.py > gpurun_out/r4l_kernels.log 2>&1; echo "kernels rc=$?"; tail -5 gpurun_out/r4l_kernels.log
echo ALL_DONE
