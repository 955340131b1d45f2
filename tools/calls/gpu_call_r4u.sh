# round 4 (u): C4 combined knobs A/B (bf16 dgrad one barrier per chunk + staggered split + 2 blocks/CU ConvT GEMMs)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for r in 1 2 3; do for v in "CDM_HALO_ONEB_BWD=0" "CDM_HALO_ONEB_BWD=1 CDM_HALO_STAGGER=1 CDM_GEMM_MINB=2"; do
  tag=$(echo $v | tr -d ' =_A-Z'); env $v timeout -k 10 300 python -u tools/train_profile.py --math bf16 > gpurun_out/r4u_c4_${tag}_$r.txt 2>&1 || { echo "$v failed"; tail -5 gpurun_out/r4u_c4_${tag}_$r.txt; exit 1; }; echo "C4 $v run $r: $(tail -1 gpurun_out/r4u_c4_${tag}_$r.txt)"; done; done
echo ALL_DONE
