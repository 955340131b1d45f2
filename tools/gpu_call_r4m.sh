# round 4 (m): trajectory tests with the on-host reference; C4 wgrad KS=4 A/B; C4 PMC families
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
CDM_PARITY_OUT=gpurun_out/r4m_parity.jsonl timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread -s tests/test_gpu_sampler.py -k "T1500 or nf128" > gpurun_out/r4m_sampler.log 2>&1; echo "sampler rc=$?"
grep -E "PASS|FAIL|Error|assert|w=" gpurun_out/r4m_sampler.log | cut -c1-400 | head -30
for r in 1 2; do for k in 0 1; do CDM_WGRAD_KS4=$k timeout -k 10 300 python -u tools/train_profile.py --math bf16 > gpurun_out/r4m_c4_ks4_${k}_$r.txt 2>&1 || { echo "ks4=$k failed"; tail -5 gpurun_out/r4m_c4_ks4_${k}_$r.txt; exit 1; }; echo "ks4=$k run $r: $(tail -1 gpurun_out/r4m_c4_ks4_${k}_$r.txt)"; done; done
timeout -k 10 300 python -u tools/train_profile.py > gpurun_out/r4m_c2.txt 2>&1 && echo "c2: $(tail -1 gpurun_out/r4m_c2.txt)"
CDM_WGRAD_KS4=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_c4_e2e.py tests/test_gpu_configs.py -k "c4" > gpurun_out/r4m_c4_ks4_tests.log 2>&1; echo "c4 tests ks4=1 rc=$?"; tail -3 gpurun_out/r4m_c4_ks4_tests.log
bash tools/pmc_step.sh gpurun_out/r4m_pmc_c4 --math bf16 > gpurun_out/r4m_pmc_c4.txt 2>&1 && echo "c4 pmc ok" || { echo "c4 pmc failed"; tail -5 gpurun_out/r4m_pmc_c4.txt; }
echo ALL_DONE
