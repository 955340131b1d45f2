# round 5 (ad): persistent two-deep ConvT GEMMs — bit-identity (multi-tile blocks vs one tile per block vs gemm_x3),
# the ConvT kernel tests, then per-kernel timing in the train step and a same-box A/B
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r5ad
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "convT" > gpurun_out/r5ad/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r5ad/tests.log
[ $rc -eq 0 ] || exit 1
for p in 1 0; do
  CDM_DEEP_PERSIST=$p timeout -k 10 400 bash tools/train_step_profile.sh gpurun_out/r5ad/prof_$p > /dev/null 2>&1 || exit 1
  echo "persist=$p"; grep -i "gemm_deep\|kernel sum" gpurun_out/r5ad/prof_$p/breakdown.txt
done
for d in 1 0 1 0; do
  CDM_DEEP_PERSIST=$d timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --cfg-sample-steps 0 --no-cpu --no-extra > gpurun_out/r5ad/ab_$d.json 2>/dev/null || exit 1
  python3 -c "import json,sys; b=json.load(open('gpurun_out/r5ad/ab_$d.json')); print('persist=$d', 'train ms', b['ms_per_step'], 'sample ms', b['sample']['ms_per_denoise_step'])" | tee -a gpurun_out/r5ad/ab.txt
done
echo ALL_DONE
