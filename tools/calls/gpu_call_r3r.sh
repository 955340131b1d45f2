# stats_mm with 8 loads in flight: standalone timing, model / bench-shape / trainer parity
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 120 python tools/row_probe.py | tee gpurun_out/r3r_probe.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_c2_e2e.py tests/test_gpu_trainer.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3r_tests.log 2>&1 || { tail -30 gpurun_out/r3r_tests.log; exit 1; }
tail -2 gpurun_out/r3r_tests.log
echo ALL_DONE
