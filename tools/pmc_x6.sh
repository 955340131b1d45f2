#!/bin/bash
# PMC passes (one counter group per pass, kernel-trace only) on the dominant conv in a given arithmetic.
#   bash tools/pmc_x6.sh [x6|h3|x3|x1|-1] [outdir]      (run from the repo root on the GPU box)
set -e
MODE=${1:-x6}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/${2:-gpurun_out/pmc_$MODE}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
         "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_MFMA" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" \
         "SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_COEXEC_CYCLES" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $C --output-format csv -d $OUT/p$i -o conv -- python3 $R/tools/conv_only.py 5 $MODE > /dev/null 2>&1 || { echo "pass $i ($C) failed"; exit 1; }
done
python3 $R/tools/pmc_summary.py $OUT > $OUT/summary.json
cat $OUT/summary.json
