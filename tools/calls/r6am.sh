# round 6 (am): the next chunk's halo staged over the last two kernel rows ($CDM_HALO_HSPLIT=1: half the pieces in row 1,
# half in row 2, same stagger halves) — bit-exactness of whole train steps (h3), then same-box A/B: sampling, C2
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6am; T=/tmp/r6am; mkdir -p $T
CDM_HALO_HSPLIT=0 timeout -k 10 200 python3 tools/tall_check.py --math h3 --out $T/a.npz || exit 1
CDM_HALO_HSPLIT=1 timeout -k 10 200 python3 tools/tall_check.py --math h3 --out $T/b.npz || exit 1
python3 tools/tall_check.py --cmp $T/a.npz $T/b.npz | tee gpurun_out/r6am/bitexact.txt
for r in 1 2 3; do
  for E in 0 1; do
    CDM_HALO_HSPLIT=$E timeout -k 10 200 python3 tools/sample_profile.py --steps 200 2>/dev/null | tail -1 | sed "s/^/hsplit=$E w0: /" | tee -a gpurun_out/r6am/ab.txt
    CDM_HALO_HSPLIT=$E timeout -k 10 200 python3 tools/train_profile.py --math h3 --steps 10 --warmup 3 2>/dev/null | tail -1 | sed "s/^/hsplit=$E C2: /" | tee -a gpurun_out/r6am/ab.txt
  done
done
echo ALL_DONE
