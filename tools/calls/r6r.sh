# round 6 (r): per-kernel A/B of the weight-gradient schedule — C2 and C4 train-step kernel traces under
# CDM_WGRAD_STAGGER=0 and 1 on one box (two rounds each), to pick the schedule per kernel variant
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6r
for r in 1 2; do
  for S in 0 1; do
    CDM_WGRAD_STAGGER=$S bash tools/train_step_profile.sh gpurun_out/r6r/c2_s${S}_$r > /dev/null 2>&1 || { echo "c2 trace failed"; exit 1; }
    CDM_WGRAD_STAGGER=$S bash tools/train_step_profile.sh gpurun_out/r6r/c4_s${S}_$r --math bf16 > /dev/null 2>&1 || { echo "c4 trace failed"; exit 1; }
    head -1 gpurun_out/r6r/c2_s${S}_$r/breakdown.txt | sed "s/^/c2 s$S r$r: /"; head -1 gpurun_out/r6r/c4_s${S}_$r/breakdown.txt | sed "s/^/c4 s$S r$r: /"
    rm -f gpurun_out/r6r/c*_s${S}_$r/sequence.txt
  done
done
echo ALL_DONE
