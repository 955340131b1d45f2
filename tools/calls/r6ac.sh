# round 6 (ac): 64-pixel K steps for the h3 row weight gradient on the 64^2 layers ($CDM_WGRAD_KS4H3=1: 133 KiB of LDS,
# 254 VGPRs) — kernel tests and C2 end-to-end parity with it on, then same-box A/B of C2 train steps
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6ac
CDM_WGRAD_KS4H3=1 timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_c2_e2e.py > gpurun_out/r6ac/tests.log 2>&1 || { echo tests failed; tail -8 gpurun_out/r6ac/tests.log; exit 1; }; tail -1 gpurun_out/r6ac/tests.log
for r in 1 2 3; do
  for E in 0 1; do
    CDM_WGRAD_KS4H3=$E timeout -k 10 200 python3 tools/train_profile.py --math h3 --steps 10 --warmup 3 2>/dev/null | tail -1 | sed "s/^/ks4h3=$E C2: /" | tee -a gpurun_out/r6ac/ab.txt
  done
done
echo ALL_DONE
