# round 5 (y): the ConvT 2x2 forward on the two-deep prefetch GEMM — bit-identity vs gemm_x3 (h3, bf16), parity of
# the e2e / sampler suites, then the sampling step's per-launch trace and a same-box A/B of the bench legs
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r5y
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_sampler.py tests/test_gpu_c2_e2e.py tests/test_gpu_c4_e2e.py > gpurun_out/r5y_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/r5y_tests.log
[ $rc -eq 0 ] || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5y -o sample -- \
    python3 tools/sample_profile.py --steps 40 > gpurun_out/r5y/sample.log 2> gpurun_out/r5y/sample.err; echo "prof rc=$?"
f=$(ls gpurun_out/r5y/*kernel_trace.csv | head -1)
python3 tools/kseg.py $f denoise_kernel 20 > gpurun_out/r5y/kseg.txt && head -8 gpurun_out/r5y/kseg.txt
python3 tools/kstep_list.py $f > gpurun_out/r5y/one_step.txt && grep -i "gemm" gpurun_out/r5y/one_step.txt; rm -f $f
for d in 1 0 1 0; do
  CDM_CONVT_DEEP=$d timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --sample-steps 200 --cfg-sample-steps 0 --no-cpu --no-extra > gpurun_out/r5y/ab_$d.json 2>/dev/null || exit 1
  python3 -c "import json,sys; b=json.load(open('gpurun_out/r5y/ab_$d.json')); print('deep=$d', 'train ms', b['ms_per_step'], 'sample ms', b['sample']['ms_per_denoise_step'])" | tee -a gpurun_out/r5y/ab.txt
done
echo ALL_DONE
