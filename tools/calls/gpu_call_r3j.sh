R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_blocks.py -x -q --timeout 200 --timeout-method thread 2>&1 | tail -15
