# round 4 (b): per-step local eps errors along the T=1500 trajectory; input-gradient tests
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
CDM_PARITY_OUT=gpurun_out/r4b_parity.jsonl timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_input_grads.py -s > gpurun_out/r4b_tests.log 2>&1; echo "tests rc=$?"
grep -E "PASS|FAIL|Error|assert|\{'x'" gpurun_out/r4b_tests.log | head -40
timeout -k 10 900 python -u tools/t1500_steps.py --w 0 --window 100 > gpurun_out/r4b_steps_w0.txt 2>&1 || { tail -30 gpurun_out/r4b_steps_w0.txt; exit 1; }
cat gpurun_out/r4b_steps_w0.txt
echo ALL_DONE
