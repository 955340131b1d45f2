# round 4 (m): trajectory tests with the on-host reference; C4 wgrad KS=4 and dy-store A/B; C4 PMC families
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "bn_bwd_fused or embed or cout1" > gpurun_out/r4m_kernels.log 2>&1; echo "kernels rc=$?"; tail -3 gpurun_out/r4m_kernels.log
CDM_PARITY_OUT=gpurun_out/r4m_parity.jsonl timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread -s tests/test_gpu_sampler.py -k "T1500 or nf128" > gpurun_out/r4m_sampler.log 2>&1; echo "sampler rc=$?"
grep -E "PASS|FAIL|Error|assert|w=" gpurun_out/r4m_sampler.log | cut -c1-400 | head -30
for r in 1 2; do for v in "CDM_WGRAD_KS4=0 CDM_DY_STORE=0" "CDM_WGRAD_KS4=1 CDM_DY_STORE=0" "CDM_WGRAD_KS4=0 CDM_DY_STORE=1" "CDM_WGRAD_KS4=1 CDM_DY_STORE=1"; do
  tag=$(echo $v | tr -d ' =_A-Z' ); env $v timeout -k 10 300 python -u tools/train_profile.py --math bf16 > gpurun_out/r4m_c4_${tag}_$r.txt 2>&1 || { echo "$v failed"; tail -5 gpurun_out/r4m_c4_${tag}_$r.txt; exit 1; }; echo "C4 $v run $r: $(tail -1 gpurun_out/r4m_c4_${tag}_$r.txt)"; done; done
for r in 1 2; do for d in 0 1; do CDM_DY_STORE=$d timeout -k 10 300 python -u tools/train_profile.py > gpurun_out/r4m_c2_dy${d}_$r.txt 2>&1 || { echo "c2 dy=$d failed"; tail -5 gpurun_out/r4m_c2_dy${d}_$r.txt; exit 1; }; echo "C2 dy=$d run $r: $(tail -1 gpurun_out/r4m_c2_dy${d}_$r.txt)"; done; done
CDM_WGRAD_KS4=1 CDM_DY_STORE=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_c4_e2e.py > gpurun_out/r4m_c4_e2e_new.log 2>&1; echo "c4 e2e ks4+dy rc=$?"; grep -E "C4 step|passed|failed" gpurun_out/r4m_c4_e2e_new.log
CDM_DY_STORE=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_c2_e2e.py > gpurun_out/r4m_c2_e2e_dy.log 2>&1; echo "c2 e2e dy rc=$?"; tail -2 gpurun_out/r4m_c2_e2e_dy.log
echo ALL_DONE
