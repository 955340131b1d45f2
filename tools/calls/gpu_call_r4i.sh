# round 4 (i): schedule host-dependence check + sampler golden tests on the golden's schedule
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
CDM_PARITY_OUT=gpurun_out/r4i_parity.jsonl timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s tests/test_gpu_sampler.py > gpurun_out/r4i_sampler.log 2>&1; echo "sampler rc=$?"
grep -E "PASS|FAIL|Error|assert|T=1500|nf=128|schedule entries" gpurun_out/r4i_sampler.log | head -40
CDM_PARITY_OUT=gpurun_out/r4i_parity.jsonl timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s tests/test_gpu_configs.py -k "sampler or T1500" > gpurun_out/r4i_cfg.log 2>&1; echo "configs rc=$?"
grep -E "PASS|FAIL|Error|assert|w=" gpurun_out/r4i_cfg.log | head -40
echo ALL_DONE
