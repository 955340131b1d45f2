# round 6 (d): epilogue cost of the roofline conv (ablation bit 16384) on the new build; the bf16 in_channels dt bar,
# the branch-pinned heights test, the train-mode input gradients without the h3 floor
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6d
T16=$((16 << 16))
A=""; for a in 1 3 5 9 16385 16445 61; do A="$A$((a | T16)),"; done
CDM_ABLS=${A%,} timeout -k 10 200 python3 tools/conv_ablation.py > gpurun_out/r6d/ablation.json 2> gpurun_out/r6d/ablation.err; echo "ablation rc=$?"; cat gpurun_out/r6d/ablation.json
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_in_channels.py tests/test_gpu_model.py tests/test_gpu_input_grads.py -k "bf16_c4 or heights or input_grads_vs or eval_mode or random_weights_vs_fp64" > gpurun_out/r6d/tests.log 2>&1; echo "tests rc=$?"
grep -E "dL/dt|in_channels=|H=|PASS|FAIL|passed|failed" gpurun_out/r6d/tests.log | cut -c1-300 | tail -40
echo ALL_DONE
