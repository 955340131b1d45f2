# round 6 (a): parity at the benchmarked sampling batch (n = 256 / the batched 512 CFG forward, h3 and bf16), the
# direct trajectory bar, in_channels > 1 (device shortcut range, bf16); then one profiled bench with the CFG legs on
# (round 5's rocprofv3 run aborted at the first CFG graph replay)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6a
export CDM_PARITY_OUT=$R/gpurun_out/r6a/parity.jsonl
timeout -k 10 700 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sample_bench_shape.py > gpurun_out/r6a/tests_bench_shape.log 2>&1; rc1=$?
echo "bench-shape tests rc=$rc1"; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/r6a/tests_bench_shape.log | tail -12
[ $rc1 -le 1 ] || exit 1
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sampler.py tests/test_gpu_in_channels.py > gpurun_out/r6a/tests_sampler.log 2>&1; rc2=$?
echo "sampler / in_channels tests rc=$rc2"; grep -E "FAIL|ERROR|passed|failed" gpurun_out/r6a/tests_sampler.log | tail -12
[ $rc2 -le 1 ] || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r6a/prof -o bench -- \
    python3 $R/bench.py --steps 5 --warmup 3 --sample-steps 20 --cfg-sample-steps 20 --no-cpu --no-extra \
    > gpurun_out/r6a/bench_under_rocprof.json 2> gpurun_out/r6a/prof.err; rc3=$?
echo "profiled bench (CFG legs on) rc=$rc3"; tail -5 gpurun_out/r6a/prof.err
rm -f gpurun_out/r6a/prof/bench_kernel_trace.csv
echo ALL_DONE
