# round 4 (k): sampler goldens on the golden's schedule; new band / embed kernels; C4 profile
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
CDM_PARITY_OUT=gpurun_out/r4k_parity.jsonl timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -s tests/test_gpu_sampler.py > gpurun_out/r4k_sampler.log 2>&1; echo "sampler rc=$?"
grep -E "PASS|FAIL|Error|assert|T=1500|nf=128|schedule entries" gpurun_out/r4k_sampler.log | head -40
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_model.py > gpurun_out/r4k_kernels.log 2>&1; echo "kernels rc=$?"; tail -5 gpurun_out/r4k_kernels.log
bash tools/train_step_profile.sh gpurun_out/r4k_prof_c4 --math bf16 && echo "c4 trace ok" && head -45 gpurun_out/r4k_prof_c4/breakdown.txt || { echo "c4 trace failed"; tail -5 gpurun_out/r4k_prof_c4/train.err; exit 1; }
bash tools/train_step_profile.sh gpurun_out/r4k_prof_c2 && echo "c2 trace ok" && head -60 gpurun_out/r4k_prof_c2/breakdown.txt
echo ALL_DONE
