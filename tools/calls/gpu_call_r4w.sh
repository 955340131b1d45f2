# round 4 (w): the 4-wave 128x64 one-term halo conv ($CDM_HALO_TALL): bit-exactness over whole C4 train steps, A/B
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r4w
for v in 0 1; do
  CDM_HALO_TALL=$v timeout -k 10 300 python -u tools/tall_check.py --out gpurun_out/r4w/t$v.npz --math bf16 > gpurun_out/r4w/check$v.log 2>&1 || { echo "check $v failed"; tail -20 gpurun_out/r4w/check$v.log; exit 1; }
  tail -1 gpurun_out/r4w/check$v.log
done
python tools/tall_check.py --cmp gpurun_out/r4w/t0.npz gpurun_out/r4w/t1.npz
for r in 1 2; do for v in 0 1; do
  echo -n "TALL=$v: "; CDM_HALO_TALL=$v timeout -k 10 200 python -u tools/train_profile.py --math bf16 --steps 20 --warmup 5 2>/dev/null | tail -1 || exit 1
done; done
CDM_HALO_TALL=1 bash tools/train_step_profile.sh gpurun_out/r4w/prof_c4_tall --math bf16 && head -30 gpurun_out/r4w/prof_c4_tall/breakdown.txt
echo ALL_DONE
