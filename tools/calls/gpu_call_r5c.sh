# round 5 (c): fixes from (b) — GN statistics for maps whose 128-pixel tiles span images, branch-pinned gradient bars
# (train nf64/128 and eval), denoise test on the schedule's own coefficients; then the driver's bench command
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
export CDM_PARITY_OUT=gpurun_out/r5c_parity.jsonl
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_model.py tests/test_gpu_input_grads.py tests/test_gpu_sampler.py::test_perturb_and_denoise_bit_exact > gpurun_out/r5c_tests.log 2>&1; echo "tests rc=$?"; tail -8 gpurun_out/r5c_tests.log
unset CDM_PARITY_OUT
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5c_bench.json 2> gpurun_out/r5c_bench.err; echo "bench rc=$?"; tail -c 1500 gpurun_out/r5c_bench.json
echo ALL_DONE
