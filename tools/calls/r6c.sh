# round 6 (c): the packed h3 split (4 VALU per pair) + one-instruction ReLU — full GPU suite on the new build, the bf16
# input-gradient probe (C = 1 and 3), then same-box interleaved A/B of the old and new builds (train step + sampling)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6c
export CDM_PARITY_OUT=$R/gpurun_out/r6c/parity.jsonl
timeout -k 10 900 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests --deselect tests/test_gpu_in_channels.py::test_in_channels_bf16_c4_arithmetic > gpurun_out/r6c/tests.log 2>&1; rc=$?
echo "suite rc=$rc"; tail -4 gpurun_out/r6c/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -m pytest -v -s --timeout 200 --timeout-method thread -m gpu tests/test_gpu_in_channels.py -k bf16 > gpurun_out/r6c/bf16_ic.log 2>&1; echo "bf16 in_channels rc=$?"
grep -E "worst tensors|dL/dt|in_channels=|passed|failed" gpurun_out/r6c/bf16_ic.log | cut -c1-500
for r in 1 2 3; do
  for L in old new; do
    CDM_LIB=$R/_ab/$L.so timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --sample-steps 100 --cfg-sample-steps 20 --no-cpu --no-extra > gpurun_out/r6c/ab_${L}_$r.json 2>/dev/null || exit 1
    python3 -c "import json; b=json.load(open('gpurun_out/r6c/ab_${L}_$r.json')); print('$L', 'train', b['ms_per_step'], 'median', b['train_step_stats']['median_ms'], 'sample', b['sample']['ms_per_denoise_step'], 'cfg3', b['sample']['cfg']['w=3']['ms_per_denoise_step'], 'conv', b['roofline']['launch_ms'])" | tee -a gpurun_out/r6c/ab.txt
  done
done
echo ALL_DONE
