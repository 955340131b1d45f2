# round-3 validation at HEAD: full GPU suite, smoke, default bench line
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out

timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_gputests_b.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r3_gputests_b.log; exit 1; }
tail -2 gpurun_out/r3_gputests_b.log
timeout -k 10 90 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke_b.log 2>&1 || { cat gpurun_out/r3_smoke_b.log; exit 1; }
tail -1 gpurun_out/r3_smoke_b.log
timeout -k 10 600 python -u bench.py > gpurun_out/r3_bench_b.json 2> gpurun_out/r3_bench_b.err || { tail -20 gpurun_out/r3_bench_b.err; exit 1; }
tail -c 400 gpurun_out/r3_bench_b.json
echo ALL_DONE
