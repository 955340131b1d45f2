# round 5 (z): the ConvT 2x2 forward and input gradient on the two-deep prefetch GEMM — bit-identity vs gemm_x3 (h3, bf16), parity of
# the e2e suites, then the train step's kernel breakdown and a same-box A/B of the bench legs
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r5z
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_c2_e2e.py tests/test_gpu_c4_e2e.py > gpurun_out/r5z_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/r5z_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 bash tools/train_step_profile.sh gpurun_out/r5z/prof; echo "prof rc=$?"
grep -i "gemm\|kernel sum" gpurun_out/r5z/prof/breakdown.txt
for d in 1 0 1 0; do
  CDM_CONVT_DEEP=$d timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --sample-steps 100 --cfg-sample-steps 0 --no-cpu --no-extra > gpurun_out/r5z/ab_$d.json 2>/dev/null || exit 1
  python3 -c "import json,sys; b=json.load(open('gpurun_out/r5z/ab_$d.json')); print('deep=$d', 'train ms', b['ms_per_step'], 'sample ms', b['sample']['ms_per_denoise_step'])" | tee -a gpurun_out/r5z/ab.txt
done
echo ALL_DONE
