# round 6 (f): block start delay (every other block of an XCD starts late) against the synchronised epilogue store
# bursts — kernel-level prod timing and bench A/B per delay (10 ns ticks)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6f
for d in 0 250 500 1000 2000; do
  echo -n "delay $d: "; CDM_HALO_DELAY=$d CDM_ABLS=$((1 | 16 << 16)) timeout -k 10 120 python3 tools/conv_ablation.py 2>/dev/null | tee -a gpurun_out/r6f/ablation.txt
done
for r in 1 2; do
  for d in 0 500 1000; do
    CDM_HALO_DELAY=$d timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --sample-steps 100 --cfg-sample-steps 0 --no-cpu --no-extra > gpurun_out/r6f/ab_${d}_$r.json 2>/dev/null || exit 1
    python3 -c "import json; b=json.load(open('gpurun_out/r6f/ab_${d}_$r.json')); print('delay $d', 'train', b['ms_per_step'], 'median', b['train_step_stats']['median_ms'], 'sample', b['sample']['ms_per_denoise_step'], 'conv', b['roofline']['launch_ms'])" | tee -a gpurun_out/r6f/ab.txt
  done
done
echo ALL_DONE
