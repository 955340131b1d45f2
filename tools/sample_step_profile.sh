#!/bin/bash
# Kernel trace + stats of the C2 sampling step: bash tools/sample_step_profile.sh <outdir> [sample_profile.py args...]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/${1:-gpurun_out/prof_sample}
shift || true
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o sample -- \
    python3 $R/tools/sample_profile.py "$@" > $OUT/sample.log 2> $OUT/sample.err
rm -f $OUT/sample_kernel_trace.csv
python3 $R/tools/kstats.py $OUT/sample_kernel_stats.csv > $OUT/summary.txt
