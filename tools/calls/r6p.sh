# round 6 (p): static priority 1 for waves 4-7 (MI355X_MICROARCH "two waves per SIMD" item 4) in the LDS-halo conv
# ($CDM_HALO_PRIO=1) and in the row weight gradient's staging-first half ($CDM_WGRAD_STAGGER=3) — the halo conv's
# timing ablations with / without, then same-box interleaved A/B of the four env settings (C2 train + sampling, C4 train)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6p
T16=$((16 << 16))
CDM_ABLS=$((1 | T16)),$((257 | T16)),$((513 | T16)),$((769 | T16)) timeout -k 10 200 python3 tools/conv_ablation.py > gpurun_out/r6p/ablation.json 2> gpurun_out/r6p/ablation.err; echo "ablation rc=$?"; cat gpurun_out/r6p/ablation.json
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --sample-steps 50 --cfg-sample-steps 0 --no-cpu --no-extra > gpurun_out/r6p/b_$tag.json 2>/dev/null || return 1
  python3 -c "import json; b=json.load(open('gpurun_out/r6p/b_$tag.json')); print('$tag', 'train', b['ms_per_step'], 'median', b['train_step_stats']['median_ms'], 'sample', b['sample']['ms_per_denoise_step'], 'conv', b['roofline']['launch_ms'])" | tee -a gpurun_out/r6p/ab.txt
  env "$@" timeout -k 10 200 python3 tools/train_profile.py --math bf16 --steps 10 --warmup 3 2>/dev/null | tail -1 | sed "s/^/$tag C4: /" | tee -a gpurun_out/r6p/ab.txt
}
for r in 1 2; do
  run base CDM_HALO_PRIO=0 || exit 1
  run hprio CDM_HALO_PRIO=1 || exit 1
  run wprio CDM_WGRAD_STAGGER=3 || exit 1
  run both CDM_HALO_PRIO=1 CDM_WGRAD_STAGGER=3 || exit 1
done
echo ALL_DONE
