# round 6 (z): the ConvT 2x2 forward with transposed accumulators and 16-byte scatter stores ($CDM_CONVT_TRO=1, one build)
# — ConvT kernel tests, whole-train-step bit-exactness against the dword-store epilogue (h3, bf16), then same-box A/B:
# sampling (w = 0, CFG), C2 / C4 train steps
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6z; T=/tmp/r6z; mkdir -p $T
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "convT" tests/test_gpu_model.py tests/test_gpu_sample_bench_shape.py > gpurun_out/r6z/tests.log 2>&1 || { echo tests failed; tail -8 gpurun_out/r6z/tests.log; exit 1; }; tail -1 gpurun_out/r6z/tests.log
for m in h3 bf16; do
  CDM_CONVT_TRO=0 timeout -k 10 200 python3 tools/tall_check.py --math $m --out $T/a_$m.npz || exit 1
  CDM_CONVT_TRO=1 timeout -k 10 200 python3 tools/tall_check.py --math $m --out $T/b_$m.npz || exit 1
  python3 tools/tall_check.py --cmp $T/a_$m.npz $T/b_$m.npz | sed "s/^/$m: /" | tee -a gpurun_out/r6z/bitexact.txt
done
for r in 1 2; do
  for E in 0 1; do
    CDM_CONVT_TRO=$E timeout -k 10 200 python3 tools/sample_profile.py --steps 200 2>/dev/null | tail -1 | sed "s/^/tro=$E w0: /" | tee -a gpurun_out/r6z/ab.txt
    CDM_CONVT_TRO=$E timeout -k 10 200 python3 tools/sample_profile.py --steps 100 --w 3 2>/dev/null | tail -1 | sed "s/^/tro=$E w3: /" | tee -a gpurun_out/r6z/ab.txt
    CDM_CONVT_TRO=$E timeout -k 10 200 python3 tools/train_profile.py --math h3 --steps 10 --warmup 3 2>/dev/null | tail -1 | sed "s/^/tro=$E C2: /" | tee -a gpurun_out/r6z/ab.txt
    CDM_CONVT_TRO=$E timeout -k 10 200 python3 tools/train_profile.py --math bf16 --steps 10 --warmup 3 2>/dev/null | tail -1 | sed "s/^/tro=$E C4: /" | tee -a gpurun_out/r6z/ab.txt
  done
done
echo ALL_DONE
