# round 6 (b): where the roofline conv's time goes (timing ablations at the shipped 16 tiles per block), the bf16
# in_channels test's per-tensor errors, the sampler bars, and the C4 step's kernel breakdown + PMC families at HEAD
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6b
T16=$((16 << 16))
A=""; for a in 1 3 5 9 13 17 21 25 29 33 45 61; do A="$A$((a | T16)),"; done
CDM_ABLS=${A%,} timeout -k 10 200 python3 tools/conv_ablation.py > gpurun_out/r6b/ablation.json 2> gpurun_out/r6b/ablation.err; echo "ablation rc=$?"; cat gpurun_out/r6b/ablation.json
timeout -k 10 400 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_in_channels.py -k "bf16 or device" tests/test_gpu_sampler.py -k "T1500 or bf16 or device" > gpurun_out/r6b/tests.log 2>&1; echo "tests rc=$?"
grep -E "worst tensors|in_channels=3|PASS|FAIL|passed|failed" gpurun_out/r6b/tests.log | cut -c1-400 | tail -20
bash tools/train_step_profile.sh gpurun_out/r6b/prof_c4 --math bf16 && echo "c4 trace ok" && head -40 gpurun_out/r6b/prof_c4/breakdown.txt || { echo "c4 trace failed"; tail -5 gpurun_out/r6b/prof_c4/train.err; exit 1; }
bash tools/pmc_step.sh gpurun_out/r6b/pmc_c4 --math bf16 > gpurun_out/r6b/pmc_c4.txt 2>&1 && echo "c4 pmc ok" || { echo "c4 pmc failed"; tail -5 gpurun_out/r6b/pmc_c4.txt; exit 1; }
echo ALL_DONE
