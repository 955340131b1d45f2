# round 4 (g): denoise kernel vs oracle at every step index and magnitude; final error maps
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/denoise_check.py > gpurun_out/r4g_denoise.txt 2>&1 || { tail -20 gpurun_out/r4g_denoise.txt; exit 1; }
cat gpurun_out/r4g_denoise.txt
for ov in none eps; do
  if [ $ov = none ]; then args=""; else args="--override $ov"; fi
  timeout -k 10 300 python -u tools/t1500_steps.py --w 0 --window 1500 $args > gpurun_out/r4g_ov_$ov.txt 2>&1 || { tail -20 gpurun_out/r4g_ov_$ov.txt; exit 1; }
  tail -4 gpurun_out/r4g_ov_$ov.txt
done
echo ALL_DONE
