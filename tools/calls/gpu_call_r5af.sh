# round 5 (af): ConvT 2x2 forward with non-temporal output stores vs plain (same process, alternating)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python3 tools/convT_probe.py > gpurun_out/r5af_convT_nt.jsonl && cat gpurun_out/r5af_convT_nt.jsonl
echo ALL_DONE
