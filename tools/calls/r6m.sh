# round 6 (m): the staggered weight-gradient schedule with the staging-first wave loading one K step further ahead
# ($CDM_WGRAD_STAGGER=1) — bit-exactness of whole C4 / C2 train steps against the lock-step schedule, then same-box
# interleaved A/B (env knob, one build); and the MFMA accumulation-bias probe with partial sums folded in fp32 VALU
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6m
timeout -k 10 120 tools/mfma_probe/acc_bias > gpurun_out/r6m/acc_bias.jsonl; echo "probe rc=$?"; cat gpurun_out/r6m/acc_bias.jsonl
for m in bf16 h3; do
  CDM_WGRAD_STAGGER=0 timeout -k 10 200 python3 tools/tall_check.py --math $m --out gpurun_out/r6m/s0_$m.npz || exit 1
  CDM_WGRAD_STAGGER=1 timeout -k 10 200 python3 tools/tall_check.py --math $m --out gpurun_out/r6m/s1_$m.npz || exit 1
  python3 tools/tall_check.py --cmp gpurun_out/r6m/s0_$m.npz gpurun_out/r6m/s1_$m.npz | tee -a gpurun_out/r6m/bitexact.txt
done
for r in 1 2 3; do
  for S in 0 1; do
    CDM_WGRAD_STAGGER=$S timeout -k 10 200 python3 tools/train_profile.py --math bf16 --steps 10 --warmup 3 2>/dev/null | tail -1 | sed "s/^/stagger=$S C4: /" | tee -a gpurun_out/r6m/ab.txt
    CDM_WGRAD_STAGGER=$S timeout -k 10 200 python3 tools/train_profile.py --math h3 --steps 10 --warmup 3 2>/dev/null | tail -1 | sed "s/^/stagger=$S C2: /" | tee -a gpurun_out/r6m/ab.txt
  done
done
echo ALL_DONE
