# round 6 (ab): 16-pixel K steps for the h3 row weight gradient ($CDM_WGRAD_KS1=1) vs 32 (default) after the schedule
# changes — kernel-level bit-exactness is not expected (another K order); same-box A/B of C2 / C4 train steps
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6ab
for r in 1 2 3; do
  for E in 0 1; do
    CDM_WGRAD_KS1=$E timeout -k 10 200 python3 tools/train_profile.py --math h3 --steps 10 --warmup 3 2>/dev/null | tail -1 | sed "s/^/ks1=$E C2: /" | tee -a gpurun_out/r6ab/ab.txt
  done
done
echo ALL_DONE
