# round-3 PMC of the C2 (h3) training step: the roofline conv launches and every kernel family
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
bash tools/pmc_step.sh gpurun_out/pmc_c2 --math h3 > gpurun_out/pmc_c2.log 2>&1 || { tail -20 gpurun_out/pmc_c2.log; exit 1; }
tail -5 gpurun_out/pmc_c2.log
echo ALL_DONE
