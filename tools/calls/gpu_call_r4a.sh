# round 4 (a): per-intermediate accuracy of the eval forward on the T=1500 states; new tests (input grads, 3-D P(k))
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/t1500_probe.py --math h3 > gpurun_out/r4a_probe_h3.txt 2>&1 || { tail -30 gpurun_out/r4a_probe_h3.txt; exit 1; }
timeout -k 10 300 python -u tools/t1500_probe.py --math fp32 > gpurun_out/r4a_probe_fp32.txt 2>&1 || { tail -30 gpurun_out/r4a_probe_fp32.txt; exit 1; }
cat gpurun_out/r4a_probe_h3.txt
CDM_PARITY_OUT=gpurun_out/r4a_parity.jsonl timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_input_grads.py tests/test_gpu_stats.py > gpurun_out/r4a_tests.log 2>&1 || { tail -40 gpurun_out/r4a_tests.log; exit 1; }
tail -3 gpurun_out/r4a_tests.log
echo ALL_DONE
