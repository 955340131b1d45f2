# round 4 (f): T=1500 excess — substitute eps / yO; baseline with fp64 embeddings
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for ov in none eps yO; do
  echo "=== override $ov"
  if [ $ov = none ]; then args=""; else args="--override $ov"; fi
  timeout -k 10 300 python -u tools/t1500_steps.py --w 0 --window 1500 $args > gpurun_out/r4f_ov_$ov.txt 2>&1 || { tail -20 gpurun_out/r4f_ov_$ov.txt; exit 1; }
  tail -2 gpurun_out/r4f_ov_$ov.txt
done
echo ALL_DONE
