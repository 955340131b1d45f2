# round 6 (aa): the kernel-row weight gradient's grid size after the schedule changes ($CDM_WGRAD_BLOCKS: 768 = three
# rounds of 256 CUs, the default; 512, 1024) — same-box interleaved A/B of C2 / C4 train steps
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6aa
for r in 1 2; do
  for B in 768 512 1024; do
    CDM_WGRAD_BLOCKS=$B timeout -k 10 200 python3 tools/train_profile.py --math h3 --steps 10 --warmup 3 2>/dev/null | tail -1 | sed "s/^/blocks=$B C2: /" | tee -a gpurun_out/r6aa/ab.txt
    CDM_WGRAD_BLOCKS=$B timeout -k 10 200 python3 tools/train_profile.py --math bf16 --steps 10 --warmup 3 2>/dev/null | tail -1 | sed "s/^/blocks=$B C4: /" | tee -a gpurun_out/r6aa/ab.txt
  done
done
echo ALL_DONE
