# round-3: grid-size A/Bs of the LDS-halo conv (blocks the tiles are dealt to) and the kernel-row weight gradient
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
bash tools/ab_c4.sh "CDM_HALO_BLOCKS=512" "CDM_HALO_BLOCKS=256" 2 > gpurun_out/c10_ab.txt 2>&1 || exit 1
bash tools/ab_c4.sh "CDM_WGRAD_BLOCKS=768" "CDM_WGRAD_BLOCKS=1536" 1 >> gpurun_out/c10_ab.txt 2>&1 || exit 1
bash tools/ab_c4.sh "CDM_WGRAD_BLOCKS=512" "CDM_WGRAD_BLOCKS=1024" 1 >> gpurun_out/c10_ab.txt 2>&1 || exit 1
cat gpurun_out/c10_ab.txt
echo ALL_DONE
