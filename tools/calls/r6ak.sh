# round 6 (ak): the uniform wave index + single-path MFMA loop for the one-term (bf16) weight gradients (first run: all
# plain-load addressing unchanged (the first form in (w) also changed the addressing) — per-kernel C4 trace A/B
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6ak; T=/tmp/r6ak; mkdir -p $T
CDM_LIB=$R/_ab/head.so timeout -k 10 200 python3 tools/tall_check.py --math bf16 --out $T/a.npz || exit 1
CDM_LIB=$R/_ab/uni.so timeout -k 10 200 python3 tools/tall_check.py --math bf16 --out $T/b.npz || exit 1
python3 tools/tall_check.py --cmp $T/a.npz $T/b.npz | tee gpurun_out/r6ak/bitexact.txt
for r in 1 2; do
  for L in head uni; do
    CDM_LIB=$R/_ab/$L.so bash tools/train_step_profile.sh gpurun_out/r6ak/c4_${L}_$r --math bf16 > /dev/null 2>&1 || { echo "trace failed"; exit 1; }
    rm -f gpurun_out/r6ak/c4_${L}_$r/sequence.txt
  done
done
python3 tools/kcmp.py gpurun_out/r6ak/c4_head_1,gpurun_out/r6ak/c4_head_2 gpurun_out/r6ak/c4_uni_1,gpurun_out/r6ak/c4_uni_2 100 > gpurun_out/r6ak/kcmp_c4.txt
grep -E "wgrad3x3_row|total" gpurun_out/r6ak/kcmp_c4.txt | cut -c1-170
echo ALL_DONE
