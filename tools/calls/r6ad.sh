# round 6 (ad): the ConvT 2x2 input gradient at two resident blocks per CU ($CDM_CONVT_DGRAD_MINB=2: 199 VGPRs, no
# spill; the 3-block form spills 36-50 at its 168 cap) — bit-exactness of whole train steps, per-kernel trace A/B (C2, C4)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6ad; T=/tmp/r6ad; mkdir -p $T
for m in h3 bf16; do
  CDM_CONVT_DGRAD_MINB=3 timeout -k 10 200 python3 tools/tall_check.py --math $m --out $T/a_$m.npz || exit 1
  CDM_CONVT_DGRAD_MINB=2 timeout -k 10 200 python3 tools/tall_check.py --math $m --out $T/b_$m.npz || exit 1
  python3 tools/tall_check.py --cmp $T/a_$m.npz $T/b_$m.npz | sed "s/^/$m: /" | tee -a gpurun_out/r6ad/bitexact.txt
done
for r in 1 2; do
  for E in 3 2; do
    CDM_CONVT_DGRAD_MINB=$E bash tools/train_step_profile.sh gpurun_out/r6ad/c2_${E}_$r > /dev/null 2>&1 || { echo "trace failed"; exit 1; }
    CDM_CONVT_DGRAD_MINB=$E bash tools/train_step_profile.sh gpurun_out/r6ad/c4_${E}_$r --math bf16 > /dev/null 2>&1 || { echo "trace failed"; exit 1; }
    rm -f gpurun_out/r6ad/c*_${E}_$r/sequence.txt
  done
done
python3 tools/kcmp.py gpurun_out/r6ad/c2_3_1,gpurun_out/r6ad/c2_3_2 gpurun_out/r6ad/c2_2_1,gpurun_out/r6ad/c2_2_2 100 > gpurun_out/r6ad/kcmp_c2.txt
python3 tools/kcmp.py gpurun_out/r6ad/c4_3_1,gpurun_out/r6ad/c4_3_2 gpurun_out/r6ad/c4_2_1,gpurun_out/r6ad/c4_2_2 100 > gpurun_out/r6ad/kcmp_c4.txt
grep -E "Gather|total" gpurun_out/r6ad/kcmp_c2.txt gpurun_out/r6ad/kcmp_c4.txt | cut -c1-200
echo ALL_DONE
