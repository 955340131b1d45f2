# round 5 (a): trajectory input audit + kink audit + the GPU suite at the round-4 state (plus the new tests)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/traj_diag.py compare > gpurun_out/r5a_traj.json 2> gpurun_out/r5a_traj.err; echo "traj rc=$?"
timeout -k 10 300 python -u tools/kink_diag.py 0,1,2,8 fp32,h3 > gpurun_out/r5a_kink.jsonl 2> gpurun_out/r5a_kink.err; echo "kink rc=$?"
CDM_PARITY_OUT=gpurun_out/r5a_parity.jsonl timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r5a_tests.log 2>&1; echo "tests rc=$?"; tail -5 gpurun_out/r5a_tests.log
echo ALL_DONE
