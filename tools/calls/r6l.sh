# round 6 (l): the bf16 weight gradient also on buffer loads, keeping its branch-form staging transforms (the selects
# were the suspected cost when (h) measured bf16 slower) — kernel / model / C4 parity, then same-box A/B wg vs bfb on C4
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6l
export CDM_PARITY_OUT=$R/gpurun_out/r6l/parity.jsonl
timeout -k 10 900 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_c4_e2e.py tests/test_gpu_in_channels.py > gpurun_out/r6l/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/r6l/tests.log
[ $rc -eq 0 ] || exit 1
for r in 1 2 3; do
  for L in wg bfb; do
    CDM_LIB=$R/_ab/$L.so timeout -k 10 200 python3 tools/train_profile.py --math bf16 --steps 10 --warmup 3 2>/dev/null | tail -1 | sed "s/^/$L C4: /" | tee -a gpurun_out/r6l/ab.txt
  done
done
echo ALL_DONE
