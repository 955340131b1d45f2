# round 5 (ae): PMC passes on the ConvT 2x2 forward (two-deep GEMM) at the bench shape — what bounds it
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 bash tools/pmc_convT.sh gpurun_out/r5ae; echo "pmc rc=$?"
echo ALL_DONE
