# round 6 (w): the row weight gradient with a provably uniform wave index and one MFMA block on a single path (the
# staggered schedule had put the K-step position in VGPRs: readfirstlane waterfall loops around every buffer load, and
# 96 accumulator copies per step at the branch joins) — kernel-level and whole-step bit-exactness vs HEAD (ct2), then
# per-kernel trace A/B (C2, C4); final form: h3 only (UNI), the one-term forms unchanged
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6w; T=/tmp/r6w; mkdir -p $T
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_c2_e2e.py tests/test_gpu_c4_e2e.py > gpurun_out/r6w/tests.log 2>&1 || { echo tests failed; tail -5 gpurun_out/r6w/tests.log; exit 1; }; tail -1 gpurun_out/r6w/tests.log
CDM_LIB=$R/_ab/ct2.so timeout -k 10 200 python3 tools/wgrad_sched_check.py --out $T/k0.npz || exit 1
CDM_LIB=$R/_ab/uw.so timeout -k 10 200 python3 tools/wgrad_sched_check.py --out $T/k1.npz || exit 1
python3 tools/wgrad_sched_check.py --cmp $T/k0.npz $T/k1.npz | tee gpurun_out/r6w/bitexact.txt
for m in h3 bf16; do
  CDM_LIB=$R/_ab/ct2.so timeout -k 10 200 python3 tools/tall_check.py --math $m --out $T/a_$m.npz || exit 1
  CDM_LIB=$R/_ab/uw.so timeout -k 10 200 python3 tools/tall_check.py --math $m --out $T/b_$m.npz || exit 1
  python3 tools/tall_check.py --cmp $T/a_$m.npz $T/b_$m.npz | sed "s/^/$m: /" | tee -a gpurun_out/r6w/bitexact.txt
done
for r in 1 2; do
  for L in ct2 uw; do
    CDM_LIB=$R/_ab/$L.so bash tools/train_step_profile.sh gpurun_out/r6w/c2_${L}_$r > /dev/null 2>&1 || { echo "trace failed"; exit 1; }
    CDM_LIB=$R/_ab/$L.so bash tools/train_step_profile.sh gpurun_out/r6w/c4_${L}_$r --math bf16 > /dev/null 2>&1 || { echo "trace failed"; exit 1; }
    head -1 gpurun_out/r6w/c2_${L}_$r/breakdown.txt | sed "s/^/c2 $L r$r: /"; head -1 gpurun_out/r6w/c4_${L}_$r/breakdown.txt | sed "s/^/c4 $L r$r: /"
    rm -f gpurun_out/r6w/c*_${L}_$r/sequence.txt
  done
done
python3 tools/kcmp.py gpurun_out/r6w/c2_ct2_1,gpurun_out/r6w/c2_ct2_2 gpurun_out/r6w/c2_uw_1,gpurun_out/r6w/c2_uw_2 100 > gpurun_out/r6w/kcmp_c2.txt
python3 tools/kcmp.py gpurun_out/r6w/c4_ct2_1,gpurun_out/r6w/c4_ct2_2 gpurun_out/r6w/c4_uw_1,gpurun_out/r6w/c4_uw_2 100 > gpurun_out/r6w/kcmp_c4.txt
grep -E "wgrad3x3_row|total" gpurun_out/r6w/kcmp_c2.txt gpurun_out/r6w/kcmp_c4.txt | cut -c1-200
echo ALL_DONE
