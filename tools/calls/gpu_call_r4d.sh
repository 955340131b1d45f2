# round 4 (d): locate the T=1500 excess by substituting fp64 reference values at stages of the HIP forward
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for ov in emb x0 x0,d1,d2 u3 x0,d1,d2,emb,film2,u3; do
  echo "=== override $ov"
  timeout -k 10 300 python -u tools/t1500_steps.py --w 0 --window 1500 --override $ov > gpurun_out/r4d_ov_$ov.txt 2>&1 || { tail -20 gpurun_out/r4d_ov_$ov.txt; exit 1; }
  tail -2 gpurun_out/r4d_ov_$ov.txt
done
echo ALL_DONE
