#!/bin/bash
# PMC passes (one counter group per pass, kernel-trace only) on the ConvT 2x2 forward (tools/convT_only.py)
#   bash tools/pmc_convT.sh [outdir]      (run from the repo root on the GPU box)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/${1:-gpurun_out/pmc_convT}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
         "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_MFMA" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $C --output-format csv -d $OUT/p$i -o conv -- python3 $R/tools/convT_only.py 5 > /dev/null 2>&1 || { echo "pass $i ($C) failed"; exit 1; }
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o conv -- python3 $R/tools/convT_only.py 20 > /dev/null 2>&1 || { echo "trace failed"; exit 1; }
python3 $R/tools/pmc_summary.py $OUT > $OUT/summary.json
cat $OUT/summary.json
grep -i gemm_deep $OUT/trace/conv_kernel_stats.csv | cut -c1-300
