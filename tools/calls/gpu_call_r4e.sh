# round 4 (e): stage substitutions (T=1500 excess) + DDP host-enqueue probe + new tests
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ddp_host_probe.py gpurun_out/r4_ddp_host_probe.json > gpurun_out/r4e_ddp.txt 2>&1 || { tail -30 gpurun_out/r4e_ddp.txt; exit 1; }
cat gpurun_out/r4e_ddp.txt
CDM_PARITY_OUT=gpurun_out/r4e_parity.jsonl timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread -s tests/test_gpu_input_grads.py tests/test_gpu_c2_e2e.py tests/test_gpu_c4_e2e.py tests/test_gpu_trainer.py tests/test_gpu_stats.py > gpurun_out/r4e_tests.log 2>&1; echo "tests rc=$?"
grep -E "PASS|FAIL|C2 step|C4 step|Error|assert" gpurun_out/r4e_tests.log | head -60
echo ALL_DONE
