set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
rocprofv3 -L > $R/gpurun_out/pmc/counters.txt 2>&1 || true
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS" ; do
  n=$(echo $C | cut -d' ' -f1)
  timeout -k 10 120 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/pmc/$n -o conv -- python3 $R/tools/conv_only.py 5 x6 > /dev/null 2>&1 || echo "pass $n failed"
done
ls -R $R/gpurun_out/pmc | head -30
