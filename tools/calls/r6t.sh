# round 6 (t): sampling-only A/B of $CDM_HALO_BEARLY (the eval forward convs: w = 0 at n = 256, CFG w = 3 at 512),
# 3 interleaved rounds on one box
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6t
for r in 1 2 3; do
  for E in 0 1; do
    CDM_HALO_BEARLY=$E timeout -k 10 200 python3 tools/sample_profile.py --steps 200 2>/dev/null | tail -1 | sed "s/^/bearly=$E w0: /" | tee -a gpurun_out/r6t/ab.txt
    CDM_HALO_BEARLY=$E timeout -k 10 200 python3 tools/sample_profile.py --steps 100 --w 3 2>/dev/null | tail -1 | sed "s/^/bearly=$E w3: /" | tee -a gpurun_out/r6t/ab.txt
  done
done
echo ALL_DONE
