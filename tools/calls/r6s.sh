# round 6 (s): the three-barrier halo schedule fetching B of the next chunk's first kernel row one group earlier
# ($CDM_HALO_BEARLY=1) — whole-train-step bit-exactness (h3), then same-box interleaved A/B: the dominant conv alone
# (tools/conv_ablation.py "prod"), C2 train + sampling (bench.py short), C4 train
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6s; T=/tmp/r6s; mkdir -p $T
CDM_HALO_BEARLY=0 timeout -k 10 200 python3 tools/tall_check.py --math h3 --out $T/a.npz || exit 1
CDM_HALO_BEARLY=1 timeout -k 10 200 python3 tools/tall_check.py --math h3 --out $T/b.npz || exit 1
python3 tools/tall_check.py --cmp $T/a.npz $T/b.npz | tee gpurun_out/r6s/bitexact.txt
for r in 1 2; do
  for E in 0 1; do
    CDM_ABLS=1 CDM_HALO_BEARLY=$E timeout -k 10 200 python3 tools/conv_ablation.py 2>/dev/null | sed "s/^/bearly=$E conv: /" | tee -a gpurun_out/r6s/ab.txt
    CDM_HALO_BEARLY=$E timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --sample-steps 100 --cfg-sample-steps 0 --no-cpu --no-extra > gpurun_out/r6s/b_$E.json 2>/dev/null || exit 1
    python3 -c "import json; b=json.load(open('gpurun_out/r6s/b_$E.json')); print('bearly=$E', 'train', b['ms_per_step'], 'median', b['train_step_stats']['median_ms'], 'sample', b['sample']['ms_per_denoise_step'], 'conv', b['roofline']['launch_ms'])" | tee -a gpurun_out/r6s/ab.txt
    CDM_HALO_BEARLY=$E timeout -k 10 200 python3 tools/train_profile.py --math bf16 --steps 10 --warmup 3 2>/dev/null | tail -1 | sed "s/^/bearly=$E C4: /" | tee -a gpurun_out/r6s/ab.txt
  done
done
echo ALL_DONE
