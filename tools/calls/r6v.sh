# round 6 (v): the ConvT 2x2 weight gradient with two register sets (the K step two ahead in flight) — ConvT kernel
# tests + C2 e2e, whole-train-step bit-exactness against HEAD's build (h3, bf16), then per-kernel trace A/B (C2, C4)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6v; T=/tmp/r6v; mkdir -p $T
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "convT" tests/test_gpu_c2_e2e.py > gpurun_out/r6v/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/r6v/tests.log; [ $rc -eq 0 ] || exit 1
for m in h3 bf16; do
  CDM_LIB=$R/_ab/head.so timeout -k 10 200 python3 tools/tall_check.py --math $m --out $T/a_$m.npz || exit 1
  CDM_LIB=$R/_ab/ct2.so timeout -k 10 200 python3 tools/tall_check.py --math $m --out $T/b_$m.npz || exit 1
  python3 tools/tall_check.py --cmp $T/a_$m.npz $T/b_$m.npz | sed "s/^/$m: /" | tee -a gpurun_out/r6v/bitexact.txt
done
for r in 1 2; do
  for L in head ct2; do
    CDM_LIB=$R/_ab/$L.so bash tools/train_step_profile.sh gpurun_out/r6v/c2_${L}_$r > /dev/null 2>&1 || { echo "trace failed"; exit 1; }
    CDM_LIB=$R/_ab/$L.so bash tools/train_step_profile.sh gpurun_out/r6v/c4_${L}_$r --math bf16 > /dev/null 2>&1 || { echo "trace failed"; exit 1; }
    head -1 gpurun_out/r6v/c2_${L}_$r/breakdown.txt | sed "s/^/c2 $L r$r: /"; head -1 gpurun_out/r6v/c4_${L}_$r/breakdown.txt | sed "s/^/c4 $L r$r: /"
    rm -f gpurun_out/r6v/c*_${L}_$r/sequence.txt
  done
done
python3 tools/kcmp.py gpurun_out/r6v/c2_head_1,gpurun_out/r6v/c2_head_2 gpurun_out/r6v/c2_ct2_1,gpurun_out/r6v/c2_ct2_2 100 > gpurun_out/r6v/kcmp_c2.txt
python3 tools/kcmp.py gpurun_out/r6v/c4_head_1,gpurun_out/r6v/c4_head_2 gpurun_out/r6v/c4_ct2_1,gpurun_out/r6v/c4_ct2_2 100 > gpurun_out/r6v/kcmp_c4.txt
grep -E "tr_x3|total" gpurun_out/r6v/kcmp_c2.txt gpurun_out/r6v/kcmp_c4.txt
echo ALL_DONE
