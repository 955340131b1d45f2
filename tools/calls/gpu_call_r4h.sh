# round 4 (h): bf16 activations (C4) — kernel tests + C4 parity + C4 timing A/B; denoise check; input grads etc.
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/denoise_check.py > gpurun_out/r4h_denoise.txt 2>&1; echo "denoise rc=$?"; cat gpurun_out/r4h_denoise.txt | tail -5
CDM_PARITY_OUT=gpurun_out/r4h_parity.jsonl timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -s tests/test_gpu_configs.py -k c4 > gpurun_out/r4h_c4tests.log 2>&1; echo "c4 tests rc=$?"
grep -E "PASS|FAIL|Error|assert|hip |grad" gpurun_out/r4h_c4tests.log | head -30
CDM_PARITY_OUT=gpurun_out/r4h_parity.jsonl timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -s tests/test_gpu_c4_e2e.py > gpurun_out/r4h_c4e2e.log 2>&1; echo "c4 e2e rc=$?"
grep -E "PASS|FAIL|Error|C4 step|assert" gpurun_out/r4h_c4e2e.log | head -20
for a in 0 1; do CDM_ACT16=$a timeout -k 10 300 python -u tools/train_profile.py --math bf16 > gpurun_out/r4h_c4_act16_$a.txt 2>&1; echo "act16=$a rc=$?"; tail -3 gpurun_out/r4h_c4_act16_$a.txt; done
for ov in none eps; do
  if [ $ov = none ]; then args=""; else args="--override $ov"; fi
  timeout -k 10 300 python -u tools/t1500_steps.py --w 0 --window 1500 $args > gpurun_out/r4h_ov_$ov.txt 2>&1 || { tail -20 gpurun_out/r4h_ov_$ov.txt; exit 1; }
  tail -4 gpurun_out/r4h_ov_$ov.txt
done
echo ALL_DONE
