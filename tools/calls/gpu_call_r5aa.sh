# round 5 (aa): out.3's band kernel on 32-channel slabs — kernel test (vs F.conv2d, bit-identity vs 16-channel slabs)
# and the same-process timing of both forms at the bench shape
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r5aa
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "cout1 or convT" > gpurun_out/r5aa/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r5aa/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 tools/cout1_probe.py > gpurun_out/r5aa/cout1.jsonl && cat gpurun_out/r5aa/cout1.jsonl
echo ALL_DONE
