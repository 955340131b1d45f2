# round 6 (u): the row weight gradient's MFMA-first half also loading the step after next once it has staged
# ($CDM_WGRAD_STAGGER=5 vs the default 1) — kernel-level bit-exactness, then same-box A/B of C2 / C4 train steps
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6u; T=/tmp/r6u; mkdir -p $T
CDM_WGRAD_STAGGER=1 timeout -k 10 200 python3 tools/wgrad_sched_check.py --out $T/k1.npz || exit 1
CDM_WGRAD_STAGGER=5 timeout -k 10 200 python3 tools/wgrad_sched_check.py --out $T/k5.npz || exit 1
python3 tools/wgrad_sched_check.py --cmp $T/k1.npz $T/k5.npz | tee gpurun_out/r6u/bitexact.txt
for r in 1 2 3; do
  for S in 1 5; do
    CDM_WGRAD_STAGGER=$S timeout -k 10 200 python3 tools/train_profile.py --math h3 --steps 10 --warmup 3 2>/dev/null | tail -1 | sed "s/^/stagger=$S C2: /" | tee -a gpurun_out/r6u/ab.txt
    CDM_WGRAD_STAGGER=$S timeout -k 10 200 python3 tools/train_profile.py --math bf16 --steps 10 --warmup 3 2>/dev/null | tail -1 | sed "s/^/stagger=$S C4: /" | tee -a gpurun_out/r6u/ab.txt
  done
done
echo ALL_DONE
