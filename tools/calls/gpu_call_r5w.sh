# round 5 (w): the fused eval epilogue with its coefficients / shortcut inputs loaded ahead of the stores — parity
# (fused vs apply kernel, sampler trajectories, in_channels) and the sampling step's per-launch trace
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r5w
export CDM_PARITY_OUT=gpurun_out/r5w_parity.jsonl
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_model.py tests/test_gpu_sampler.py tests/test_gpu_in_channels.py > gpurun_out/r5w_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/r5w_tests.log
[ $rc -eq 0 ] || exit 1
unset CDM_PARITY_OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5w -o sample -- \
    python3 tools/sample_profile.py --steps 40 > gpurun_out/r5w/sample.log 2> gpurun_out/r5w/sample.err; echo "prof rc=$?"
f=$(ls gpurun_out/r5w/*kernel_trace.csv | head -1)
python3 tools/kseg.py $f denoise_kernel 20 > gpurun_out/r5w/kseg.txt && head -8 gpurun_out/r5w/kseg.txt
python3 tools/kstep_list.py $f > gpurun_out/r5w/one_step.txt && grep "true>" gpurun_out/r5w/one_step.txt; rm -f $f
echo ALL_DONE
