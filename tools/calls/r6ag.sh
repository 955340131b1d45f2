# round 6 (ag): halo-conv launch knobs re-checked on the sampling step after the schedule changes — $CDM_HALO_BLOCKS
# (256: one round of one block per CU, up to 16 tiles each = default; 512) and $CDM_HALO_STAGGER (h3 default 1)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6ag
for r in 1 2; do
  for V in "base" "CDM_HALO_BLOCKS=512" "CDM_HALO_STAGGER=0"; do
    if [ "$V" = base ]; then E=""; else E="$V"; fi
    env $E timeout -k 10 200 python3 tools/sample_profile.py --steps 200 2>/dev/null | tail -1 | sed "s/^/$V w0: /" | tee -a gpurun_out/r6ag/ab.txt
    env $E timeout -k 10 200 python3 tools/train_profile.py --math h3 --steps 10 --warmup 3 2>/dev/null | tail -1 | sed "s/^/$V C2: /" | tee -a gpurun_out/r6ag/ab.txt
  done
done
echo ALL_DONE
