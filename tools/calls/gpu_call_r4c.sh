# round 4 (c): per-intermediate coherent errors along the T=1500 trajectory; input-gradient seed scan; nf=128 sampler
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
CDM_PARITY_OUT=gpurun_out/r4c_parity.jsonl timeout -k 10 600 python -u -m pytest -v --timeout 400 --timeout-method thread -s tests/test_gpu_sampler.py -k "nf128 or T1500" > gpurun_out/r4c_sampler.log 2>&1; echo "sampler tests rc=$?"
grep -E "PASS|FAIL|nf=128|T=1500|Error" gpurun_out/r4c_sampler.log | head -20
timeout -k 10 900 python -u tools/t1500_steps.py --w 0 --window 250 --layers > gpurun_out/r4c_layers_w0.txt 2>&1 || { tail -30 gpurun_out/r4c_layers_w0.txt; exit 1; }
cat gpurun_out/r4c_layers_w0.txt
timeout -k 10 600 python -u tools/input_grad_seed_scan.py 10 > gpurun_out/r4c_seed_scan.txt 2>&1 || { tail -30 gpurun_out/r4c_seed_scan.txt; exit 1; }
cat gpurun_out/r4c_seed_scan.txt
echo ALL_DONE
