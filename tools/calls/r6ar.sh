# round 6 (ar): the one-barrier (bf16) halo schedule with the same branch-free last-row stores — tests, bit-exactness (bf16), same-box A/B (C4 train, bf16 sampling)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6ar; T=/tmp/r6ar; mkdir -p $T
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_c4_e2e.py > gpurun_out/r6ar/tests.log 2>&1 || { echo tests failed; tail -8 gpurun_out/r6ar/tests.log; exit 1; }; tail -1 gpurun_out/r6ar/tests.log
CDM_LIB=$R/_ab/head.so timeout -k 10 200 python3 tools/tall_check.py --math bf16 --out $T/a.npz || exit 1
CDM_LIB=$R/_ab/bf.so timeout -k 10 200 python3 tools/tall_check.py --math bf16 --out $T/b.npz || exit 1
python3 tools/tall_check.py --cmp $T/a.npz $T/b.npz | tee gpurun_out/r6ar/bitexact.txt
for r in 1 2 3; do
  for L in head bf; do
    CDM_LIB=$R/_ab/$L.so timeout -k 10 200 python3 tools/sample_profile.py --steps 200 --math bf16 2>/dev/null | tail -1 | sed "s/^/$L w0: /" | tee -a gpurun_out/r6ar/ab.txt
    CDM_LIB=$R/_ab/$L.so timeout -k 10 200 python3 tools/train_profile.py --math bf16 --steps 10 --warmup 3 2>/dev/null | tail -1 | sed "s/^/$L C4: /" | tee -a gpurun_out/r6ar/ab.txt
  done
done
echo ALL_DONE
