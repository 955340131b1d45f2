# round 4 (r): PMC passes of the C2 and C4 training steps; DDP host-enqueue probe (one-rank RCCL)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
bash tools/pmc_step.sh gpurun_out/r4_pmc_c2 > gpurun_out/r4_pmc_c2.log 2>&1 && echo "c2 pmc ok" || { echo "c2 pmc failed"; tail -5 gpurun_out/r4_pmc_c2.log; exit 1; }
bash tools/pmc_step.sh gpurun_out/r4_pmc_c4 --math bf16 > gpurun_out/r4_pmc_c4.log 2>&1 && echo "c4 pmc ok" || { echo "c4 pmc failed"; tail -5 gpurun_out/r4_pmc_c4.log; exit 1; }
timeout -k 10 400 python -u tools/ddp_host_probe.py gpurun_out/r4_ddp_host_probe.json > gpurun_out/r4_ddp.txt 2>&1; echo "ddp probe rc=$?"; tail -6 gpurun_out/r4_ddp.txt
bash tools/train_step_profile.sh gpurun_out/r4r_prof_c2 && echo "c2 trace ok" && head -3 gpurun_out/r4r_prof_c2/breakdown.txt
bash tools/train_step_profile.sh gpurun_out/r4r_prof_c4 --math bf16 && echo "c4 trace ok" && head -3 gpurun_out/r4r_prof_c4/breakdown.txt
echo ALL_DONE
