# round 6 (af): the transposed ConvT 2x2 forward now also where the bias is not 16-byte aligned (the packed parameter
# buffer: in (z) it had stayed on the dword-store epilogue in the model) — ConvT tests, bit-exactness, same-box A/B
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6af; T=/tmp/r6af; mkdir -p $T
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k convT > gpurun_out/r6af/tests.log 2>&1 || { echo tests failed; tail -8 gpurun_out/r6af/tests.log; exit 1; }; tail -1 gpurun_out/r6af/tests.log
for m in h3 bf16; do
  CDM_CONVT_TRO=0 timeout -k 10 200 python3 tools/tall_check.py --math $m --out $T/a_$m.npz || exit 1
  CDM_CONVT_TRO=1 timeout -k 10 200 python3 tools/tall_check.py --math $m --out $T/b_$m.npz || exit 1
  python3 tools/tall_check.py --cmp $T/a_$m.npz $T/b_$m.npz | sed "s/^/$m: /" | tee -a gpurun_out/r6af/bitexact.txt
done
for r in 1 2; do
  for E in 0 1; do
    CDM_CONVT_TRO=$E timeout -k 10 200 python3 tools/sample_profile.py --steps 200 2>/dev/null | tail -1 | sed "s/^/tro=$E w0: /" | tee -a gpurun_out/r6af/ab.txt
    CDM_CONVT_TRO=$E timeout -k 10 200 python3 tools/train_profile.py --math h3 --steps 10 --warmup 3 2>/dev/null | tail -1 | sed "s/^/tro=$E C2: /" | tee -a gpurun_out/r6af/ab.txt
  done
done
export TMPDIR=/tmp
for E in 0 1; do
  CDM_CONVT_TRO=$E timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6af/t$E -o s -- python3 tools/sample_profile.py --steps 20 > /dev/null 2>&1 || exit 1
  grep -h "gemm_deep" gpurun_out/r6af/t$E/s_kernel_stats.csv | cut -d, -f1-6 | sed "s/^/tro=$E: /" | tee -a gpurun_out/r6af/ab.txt
  rm -f gpurun_out/r6af/t$E/*trace.csv
done
echo ALL_DONE
