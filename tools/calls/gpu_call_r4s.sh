# round 4 (s): standalone blocks: eval-mode backward and the C_in = 1 image gradient; sampling-step kernel profile
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_blocks.py > gpurun_out/r4s_blocks.log 2>&1; echo "blocks rc=$?"; grep -E "PASS|FAIL|Error|assert" gpurun_out/r4s_blocks.log | head -40
bash tools/sample_step_profile.sh gpurun_out/r4s_prof_sample && echo "sample trace ok" && cat gpurun_out/r4s_prof_sample/sample.log | tail -2 && head -30 gpurun_out/r4s_prof_sample/summary.txt
echo ALL_DONE
