# round 6 (g): wave-uniform epilogue addressing (EpiStoreW, the row weight gradient's slab stores, the ConvT 2x2
# scatter) — full GPU suite, the epilogue ablation on the new build, same-box A/B base (packed split) vs epi
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6g
export CDM_PARITY_OUT=$R/gpurun_out/r6g/parity.jsonl
timeout -k 10 900 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r6g/tests.log 2>&1; rc=$?
echo "suite rc=$rc"; tail -3 gpurun_out/r6g/tests.log
[ $rc -eq 0 ] || exit 1
T16=$((16 << 16)); CDM_ABLS=$((1 | T16)),$((16385 | T16)) timeout -k 10 120 python3 tools/conv_ablation.py > gpurun_out/r6g/ablation.json 2>/dev/null; cat gpurun_out/r6g/ablation.json
for r in 1 2 3; do
  for L in base epi; do
    CDM_LIB=$R/_ab/$L.so timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --sample-steps 100 --cfg-sample-steps 20 --no-cpu --no-extra > gpurun_out/r6g/ab_${L}_$r.json 2>/dev/null || exit 1
    python3 -c "import json; b=json.load(open('gpurun_out/r6g/ab_${L}_$r.json')); print('$L', 'train', b['ms_per_step'], 'median', b['train_step_stats']['median_ms'], 'sample', b['sample']['ms_per_denoise_step'], 'cfg3', b['sample']['cfg']['w=3']['ms_per_denoise_step'], 'conv', b['roofline']['launch_ms'])" | tee -a gpurun_out/r6g/ab.txt
  done
done
echo ALL_DONE
