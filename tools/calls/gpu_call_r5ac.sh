# round 5 (ac): rocprofv3 kernel trace + stats of the bench at final HEAD (h3, CFG legs skipped under the profiler) and
# the PMC passes on the dominant conv (tools/gpu_profile.sh)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 1000 bash tools/gpu_profile.sh gpurun_out/r5ac h3; echo "prof rc=$?"
python3 tools/kstats.py gpurun_out/r5ac/trace/bench_kernel_stats.csv > gpurun_out/r5ac/summary.txt && head -8 gpurun_out/r5ac/summary.txt
tail -c 600 gpurun_out/r5ac/bench_under_rocprof.json
echo ALL_DONE
