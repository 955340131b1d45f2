# round 6 (e): next-chunk loads issued ahead of the epilogue stores (EARLY) — kernel / model parity on both variants,
# then same-box A/B: base (packed split) vs EARLY without / with the BN-backward dgrads
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6e
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_c2_e2e.py > gpurun_out/r6e/tests_nobwd.log 2>&1; rc=$?
echo "tests (ei_nobwd) rc=$rc"; tail -2 gpurun_out/r6e/tests_nobwd.log
[ $rc -eq 0 ] || exit 1
CDM_LIB=$R/_ab/ei_all.so timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_c2_e2e.py > gpurun_out/r6e/tests_all.log 2>&1; rc=$?
echo "tests (ei_all) rc=$rc"; tail -2 gpurun_out/r6e/tests_all.log
[ $rc -eq 0 ] || exit 1
for r in 1 2; do
  for L in base ei_nobwd ei_all; do
    CDM_LIB=$R/_ab/$L.so timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --sample-steps 100 --cfg-sample-steps 0 --no-cpu --no-extra > gpurun_out/r6e/ab_${L}_$r.json 2>/dev/null || exit 1
    python3 -c "import json; b=json.load(open('gpurun_out/r6e/ab_${L}_$r.json')); print('$L', 'train', b['ms_per_step'], 'median', b['train_step_stats']['median_ms'], 'sample', b['sample']['ms_per_denoise_step'], 'conv', b['roofline']['launch_ms'])" | tee -a gpurun_out/r6e/ab.txt
  done
done
echo ALL_DONE
