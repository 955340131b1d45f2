# round 4 (p): load-ahead accumulate epilogue (compile-time variant); A/B C2 sums-in-wgrad, C4 dy pass; tests
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_model.py > gpurun_out/r4p_kernels.log 2>&1; echo "kernels+model rc=$?"; tail -2 gpurun_out/r4p_kernels.log
for r in 1 2; do for v in "CDM_DY_PASS=0" "CDM_DY_PASS=1"; do
  tag=$(echo $v | tr -d ' =_A-Z'); env $v timeout -k 10 300 python -u tools/train_profile.py --math bf16 > gpurun_out/r4p_c4_${tag}_$r.txt 2>&1 || { echo "$v failed"; tail -5 gpurun_out/r4p_c4_${tag}_$r.txt; exit 1; }; echo "C4 $v run $r: $(tail -1 gpurun_out/r4p_c4_${tag}_$r.txt)"; done; done
for r in 1 2; do for d in 0 1; do CDM_FUSE_BN_SUMS=$d timeout -k 10 300 python -u tools/train_profile.py > gpurun_out/r4p_c2_sums${d}_$r.txt 2>&1 || { echo "c2 sums=$d failed"; tail -5 gpurun_out/r4p_c2_sums${d}_$r.txt; exit 1; }; echo "C2 CDM_FUSE_BN_SUMS=$d run $r: $(tail -1 gpurun_out/r4p_c2_sums${d}_$r.txt)"; done; done
CDM_FUSE_BN_SUMS=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_c2_e2e.py > gpurun_out/r4p_c2_e2e_sums.log 2>&1; echo "c2 e2e sums rc=$?"; tail -1 gpurun_out/r4p_c2_e2e_sums.log
bash tools/train_step_profile.sh gpurun_out/r4p_prof_c4 --math bf16 && echo "c4 trace ok" && head -3 gpurun_out/r4p_prof_c4/breakdown.txt
bash tools/train_step_profile.sh gpurun_out/r4p_prof_c2 && echo "c2 trace ok" && head -3 gpurun_out/r4p_prof_c2/breakdown.txt
echo ALL_DONE
