# round 4 (q): full GPU suite at the round's defaults, the bench (default driver command), a kernel trace of a short bench
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
CDM_PARITY_OUT=gpurun_out/r4q_parity.jsonl timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread -m gpu tests/ > gpurun_out/r4q_gpu_tests.log 2>&1; echo "gpu tests rc=$?"
grep -E "FAILED|Error|passed|failed" gpurun_out/r4q_gpu_tests.log | tail -8
timeout -k 10 900 python -u bench.py > gpurun_out/r4_bench.json 2> gpurun_out/r4_bench.err || { echo "bench failed"; tail -20 gpurun_out/r4_bench.err; exit 1; }
head -c 1200 gpurun_out/r4_bench.json; echo
bash tools/trace_bench.sh gpurun_out/r4_trace && echo "trace ok" && head -25 gpurun_out/r4_trace/summary.txt
echo ALL_DONE
