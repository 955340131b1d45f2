# round 6 (q): C2 and C4 train-step kernel breakdowns at HEAD (early-load staggered weight gradient), and the PMC
# families of both steps
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6q
bash tools/train_step_profile.sh gpurun_out/r6q/prof_c2 && echo "c2 trace ok" && head -30 gpurun_out/r6q/prof_c2/breakdown.txt || { echo "c2 trace failed"; tail -5 gpurun_out/r6q/prof_c2/train.err; exit 1; }
bash tools/train_step_profile.sh gpurun_out/r6q/prof_c4 --math bf16 && echo "c4 trace ok" && head -16 gpurun_out/r6q/prof_c4/breakdown.txt || { echo "c4 trace failed"; exit 1; }
bash tools/pmc_step.sh gpurun_out/r6q/pmc_c2 > gpurun_out/r6q/pmc_c2.txt 2>&1 && echo "c2 pmc ok" || { echo "c2 pmc failed"; tail -5 gpurun_out/r6q/pmc_c2.txt; exit 1; }
bash tools/pmc_step.sh gpurun_out/r6q/pmc_c4 --math bf16 > gpurun_out/r6q/pmc_c4.txt 2>&1 && echo "c4 pmc ok" || { echo "c4 pmc failed"; tail -5 gpurun_out/r6q/pmc_c4.txt; exit 1; }
rm -rf gpurun_out/r6q/pmc_c2/p* gpurun_out/r6q/pmc_c4/p*
echo ALL_DONE
