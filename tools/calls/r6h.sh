# round 6 (h): the row weight gradient's K-step loads as buffer loads (uniform base + step-invariant lane offsets, OOB
# zeros for padding) and branch-free staging transforms — kernel / model / e2e parity, then same-box A/B base vs wg
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6h
export CDM_PARITY_OUT=$R/gpurun_out/r6h/parity.jsonl
timeout -k 10 900 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_c2_e2e.py tests/test_gpu_c4_e2e.py tests/test_gpu_trainer.py tests/test_gpu_configs.py > gpurun_out/r6h/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/r6h/tests.log
[ $rc -eq 0 ] || exit 1
for r in 1 2 3; do
  for L in base wg; do
    CDM_LIB=$R/_ab/$L.so timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --sample-steps 100 --cfg-sample-steps 0 --no-cpu --no-extra > gpurun_out/r6h/ab_${L}_$r.json 2>/dev/null || exit 1
    python3 -c "import json; b=json.load(open('gpurun_out/r6h/ab_${L}_$r.json')); print('$L', 'train', b['ms_per_step'], 'median', b['train_step_stats']['median_ms'], 'sample', b['sample']['ms_per_denoise_step'], 'conv', b['roofline']['launch_ms'])" | tee -a gpurun_out/r6h/ab.txt
    CDM_LIB=$R/_ab/$L.so timeout -k 10 200 python3 tools/train_profile.py --math bf16 --steps 10 --warmup 3 2>/dev/null | tail -1 | sed "s/^/$L C4: /" | tee -a gpurun_out/r6h/ab.txt
  done
done
echo ALL_DONE
