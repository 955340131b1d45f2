# round-3 rocprofv3 kernel trace + stats of the bench command (short sampling; no CPU / extra legs), summarised
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
bash tools/trace_bench.sh gpurun_out/r3_trace || { tail -20 gpurun_out/r3_trace/trace.err; exit 1; }
head -25 gpurun_out/r3_trace/summary.txt
tail -c 300 gpurun_out/r3_trace/bench.json
