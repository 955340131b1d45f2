# row kernels with one memory round trip before the barrier + amax commits that skip redundant atomics:
# standalone timing, kernel / model parity, train-step A/B and trace
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
CDM_ROW_KERNELS=1 timeout -k 10 120 python tools/row_probe.py | tee gpurun_out/r3p_probe.txt
CDM_ROW_KERNELS=0 timeout -k 10 120 python tools/row_probe.py | tee -a gpurun_out/r3p_probe.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3p_tests.log 2>&1 || { tail -30 gpurun_out/r3p_tests.log; exit 1; }
tail -3 gpurun_out/r3p_tests.log
bash tools/ab_c4.sh "CDM_ROW_KERNELS=0" "CDM_ROW_KERNELS=1" 2 | tee gpurun_out/r3p_ab.txt
bash tools/train_step_profile.sh gpurun_out/r3p_prof --math h3 && head -40 gpurun_out/r3p_prof/breakdown.txt | grep -n "cin1\|cout1\|stats_mm\|kernel sum\|norm_apply"
echo ALL_DONE
