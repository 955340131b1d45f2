# validation at HEAD after the row-kernel / amax changes: standalone timing, full GPU suite, smoke, bench, C2 trace
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
CDM_ROW_KERNELS=1 timeout -k 10 120 python tools/row_probe.py | tee gpurun_out/r3f_probe.txt
CDM_ROW_KERNELS=0 timeout -k 10 120 python tools/row_probe.py | tee -a gpurun_out/r3f_probe.txt
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_gputests_f.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r3_gputests_f.log; exit 1; }
tail -2 gpurun_out/r3_gputests_f.log
timeout -k 10 90 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke_f.log 2>&1 || { cat gpurun_out/r3_smoke_f.log; exit 1; }
tail -1 gpurun_out/r3_smoke_f.log
timeout -k 10 600 python -u bench.py > gpurun_out/r3_bench_f.json 2> gpurun_out/r3_bench_f.err || { tail -20 gpurun_out/r3_bench_f.err; exit 1; }
tail -c 300 gpurun_out/r3_bench_f.json
bash tools/train_step_profile.sh gpurun_out/r3f_prof --math h3 && head -40 gpurun_out/r3f_prof/breakdown.txt | grep -n "cin1\|cout1\|stats_mm\|kernel sum\|norm_apply"
echo ALL_DONE
