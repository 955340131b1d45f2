# round 5 (x): the C2 train step's launch sequence at HEAD (per-launch durations, to find epilogue / apply stalls)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 400 bash tools/train_step_profile.sh gpurun_out/r5x; echo "prof rc=$?"
head -40 gpurun_out/r5x/breakdown.txt
echo ALL_DONE
