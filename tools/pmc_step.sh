#!/bin/bash
# PMC passes on the training step (one counter group per pass, kernel-trace only; tools/pmc_step.py selects the
# roofline conv launches).   bash tools/pmc_step.sh [outdir] [train_profile.py args, e.g. --math bf16]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/${1:-gpurun_out/pmc_step}
shift || true
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for C in "FETCH_SIZE" "WRITE_SIZE" \
         "SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d $OUT/p$i -o step -- python3 $R/tools/train_profile.py --steps 4 --warmup 3 "$@" > $OUT/p$i.log 2>&1 || { echo "pass $i ($C) failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 $R/tools/pmc_step.py $OUT > $OUT/summary.json
python3 $R/tools/pmc_families.py $OUT > $OUT/families.json
cat $OUT/summary.json
