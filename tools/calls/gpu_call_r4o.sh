# round 4 (o): accumulate epilogue, out.1 GN fused into out.3, bf16 dy pass: tests + A/B
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_model.py > gpurun_out/r4o_kernels.log 2>&1; echo "kernels+model rc=$?"; tail -3 gpurun_out/r4o_kernels.log
CDM_DY_PASS=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_c4_e2e.py tests/test_gpu_configs.py -k "c4" > gpurun_out/r4o_c4_dypass.log 2>&1; echo "c4 tests dy_pass rc=$?"; grep -E "C4 step|passed|failed" gpurun_out/r4o_c4_dypass.log | head
for r in 1 2; do for v in "CDM_DY_PASS=0 CDM_FUSE_GN_OUT=0" "CDM_DY_PASS=0 CDM_FUSE_GN_OUT=1" "CDM_DY_PASS=1 CDM_FUSE_GN_OUT=1"; do
  tag=$(echo $v | tr -d ' =_A-Z'); env $v timeout -k 10 300 python -u tools/train_profile.py --math bf16 > gpurun_out/r4o_c4_${tag}_$r.txt 2>&1 || { echo "$v failed"; tail -5 gpurun_out/r4o_c4_${tag}_$r.txt; exit 1; }; echo "C4 $v run $r: $(tail -1 gpurun_out/r4o_c4_${tag}_$r.txt)"; done; done
for r in 1 2; do for d in 0 1; do CDM_FUSE_GN_OUT=$d timeout -k 10 300 python -u tools/train_profile.py > gpurun_out/r4o_c2_gn${d}_$r.txt 2>&1 || { echo "c2 gn=$d failed"; exit 1; }; echo "C2 CDM_FUSE_GN_OUT=$d run $r: $(tail -1 gpurun_out/r4o_c2_gn${d}_$r.txt)"; done; done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_c2_e2e.py tests/test_gpu_c4_e2e.py tests/test_gpu_trainer.py > gpurun_out/r4o_e2e.log 2>&1; echo "e2e rc=$?"; tail -2 gpurun_out/r4o_e2e.log
echo ALL_DONE
