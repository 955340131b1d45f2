#!/bin/bash
# PMC passes over the h3 LDS-halo conv (128->128 @64x64, B=256) via tools/conv_ablation.py (shipped schedule only):
# wave-state split, MFMA busy, LDS activity.  Writes gpurun_out/pmc_halo/p<N>/...counter_collection.csv
set -e
export TMPDIR=/tmp CDM_ABLS=${CDM_ABLS:-524289}
OUT=${OUT:-gpurun_out/pmc_halo}
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES GRBM_COUNT"
i=0
for P in "$P1" "$P2"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex conv3x3_halo --output-format csv -d $OUT/p$i -o run -- python3 tools/conv_ablation.py > $OUT.p$i.log 2>&1
done
