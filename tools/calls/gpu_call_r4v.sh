# round 4 (v): final — full GPU suite at the round's defaults, the bench (driver command), smoke()
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
CDM_PARITY_OUT=gpurun_out/r4v_parity.jsonl timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread -m gpu tests/ > gpurun_out/r4v_gpu_tests.log 2>&1; echo "gpu tests rc=$?"
grep -E "FAILED|Error|passed|failed" gpurun_out/r4v_gpu_tests.log | tail -8
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4v_smoke.txt 2>&1; echo "smoke rc=$?"; tail -2 gpurun_out/r4v_smoke.txt
timeout -k 10 900 python -u bench.py > gpurun_out/r4v_bench.json 2> gpurun_out/r4v_bench.err || { echo "bench failed"; tail -20 gpurun_out/r4v_bench.err; exit 1; }
head -c 700 gpurun_out/r4v_bench.json; echo
echo ALL_DONE
