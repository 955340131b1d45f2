# round-3 measurement call: C4 (bf16) PMC passes, train-step kernel breakdowns (bf16, h3), RCCL API + kernel trace
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
CDM_PMC_KERNEL="conv3x3_halo_x3_kernel<1, 64," bash tools/pmc_step.sh gpurun_out/pmc_c4 --math bf16 > gpurun_out/pmc_c4.log 2>&1 || { tail -20 gpurun_out/pmc_c4.log; exit 1; }
bash tools/train_step_profile.sh gpurun_out/prof_c4 --math bf16 || exit 1
bash tools/train_step_profile.sh gpurun_out/prof_c2 --math h3 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --rccl-trace --hip-runtime-trace --output-format csv -d $R/gpurun_out/r3_rccl2 -o rccl -- python3 $R/tools/rccl_trace.py > $R/gpurun_out/rccl2.log 2>&1 || exit 1
echo ALL_DONE
