# round 4 (n): full GPU suite with dy store + KS4 defaults, eval-mode gradients; C2 / C4 step timing and traces
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
CDM_PARITY_OUT=gpurun_out/r4n_parity.jsonl timeout -k 10 1500 python -u -m pytest -v --timeout 600 --timeout-method thread -m gpu tests/ > gpurun_out/r4n_gpu_tests.log 2>&1; echo "gpu tests rc=$?"
grep -E "FAIL|Error|passed|failed" gpurun_out/r4n_gpu_tests.log | tail -15
bash tools/train_step_profile.sh gpurun_out/r4n_prof_c4 --math bf16 && echo "c4 trace ok" && head -30 gpurun_out/r4n_prof_c4/breakdown.txt
bash tools/train_step_profile.sh gpurun_out/r4n_prof_c2 && echo "c2 trace ok" && head -20 gpurun_out/r4n_prof_c2/breakdown.txt
echo ALL_DONE
