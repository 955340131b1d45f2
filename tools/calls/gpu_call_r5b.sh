# round 5 (b): the GPU suite on the parity fixes (trajectory inputs, kink branches, fp64 DFT, C4 eval under autograd,
# EmbedFC input_dim, map heights % 4), the fused eval epilogue, out.3 band prefetch, up0 on the 16-bit matrix cores,
# the batched bf16 repack; then the sampling step fused vs unfused (kernel summaries)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
export CDM_PARITY_OUT=gpurun_out/r5b_parity.jsonl
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r5b_tests.log 2>&1; echo "tests rc=$?"; tail -5 gpurun_out/r5b_tests.log
unset CDM_PARITY_OUT
bash tools/sample_step_profile.sh gpurun_out/r5b_prof_fused --steps 60 && echo fused && cat gpurun_out/r5b_prof_fused/sample.log && head -16 gpurun_out/r5b_prof_fused/summary.txt
CDM_FUSE_EVAL=0 bash tools/sample_step_profile.sh gpurun_out/r5b_prof_unfused --steps 60 && echo unfused && cat gpurun_out/r5b_prof_unfused/sample.log && head -16 gpurun_out/r5b_prof_unfused/summary.txt
echo ALL_DONE
