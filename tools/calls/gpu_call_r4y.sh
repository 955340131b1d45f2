# round 4 (y): C2 train-step kernel trace at HEAD (the balanced cout1 band kernel, the tiled embed weight gradient)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
bash tools/train_step_profile.sh gpurun_out/r4y_prof_c2 && head -60 gpurun_out/r4y_prof_c2/breakdown.txt | grep -E "steps:|cout1|embed|chan_reduce|norm_apply" 
echo ALL_DONE
