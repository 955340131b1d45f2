# round 6 (aj): per-rank cost of the data-parallel step (eager, bucketed async all-reduce in a one-rank RCCL group) vs
# the graph-replayed single-GPU step — what an N > 1 bench run pays per rank before any inter-GPU traffic
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6aj
timeout -k 10 300 python3 tools/ddp_step_probe.py 10 > gpurun_out/r6aj/probe.json 2> gpurun_out/r6aj/probe.err; echo "rc=$?"; cat gpurun_out/r6aj/probe.json; tail -3 gpurun_out/r6aj/probe.err
echo ALL_DONE
