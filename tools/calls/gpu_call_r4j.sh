# round 4 (j): C4 (bf16 activations) kernel trace breakdown + PMC families; C2 breakdown for reference
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
bash tools/train_step_profile.sh gpurun_out/r4j_prof_c4 --math bf16 && echo "c4 trace ok" && head -45 gpurun_out/r4j_prof_c4/breakdown.txt || { echo "c4 trace failed"; tail -5 gpurun_out/r4j_prof_c4/train.err; exit 1; }
bash tools/pmc_step.sh gpurun_out/r4j_pmc_c4 --math bf16 > gpurun_out/r4j_pmc_c4.txt 2>&1 && echo "c4 pmc ok" || { echo "c4 pmc failed"; tail -5 gpurun_out/r4j_pmc_c4.txt; exit 1; }
bash tools/train_step_profile.sh gpurun_out/r4j_prof_c2 && echo "c2 trace ok" && head -30 gpurun_out/r4j_prof_c2/breakdown.txt
echo ALL_DONE
