# round 5 (z2): same-box A/B of the two-deep ConvT GEMMs over the full T = 1500 sampling run and 30 train steps
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r5z2
for d in 0 1 0 1 0 1; do
  CDM_CONVT_DEEP=$d timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --cfg-sample-steps 0 --no-cpu --no-extra > gpurun_out/r5z2/ab_$d.json 2>/dev/null || exit 1
  python3 -c "import json,sys; b=json.load(open('gpurun_out/r5z2/ab_$d.json')); print('deep=$d', 'train ms', b['ms_per_step'], 'sample ms', b['sample']['ms_per_denoise_step'])" | tee -a gpurun_out/r5z2/ab.txt
done
echo ALL_DONE
