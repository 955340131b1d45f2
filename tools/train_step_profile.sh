#!/bin/bash
# Kernel trace of the C2 train step (bs=256, n_feat=128, graph-replayed) and its per-step breakdown by kernel:
#   bash tools/train_step_profile.sh <outdir> [train_profile.py args...]
# writes <outdir>/train_kernel_stats.csv (rocprofv3 --stats) and <outdir>/breakdown.txt (tools/kstep.py)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/${1:-gpurun_out/prof_train}
shift || true
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o train -- \
    python3 $R/tools/train_profile.py --steps 10 --warmup 3 "$@" > $OUT/train.log 2> $OUT/train.err
python3 $R/tools/kstep.py $OUT/train_kernel_trace.csv 8 > $OUT/breakdown.txt
python3 $R/tools/kseq.py $OUT/train_kernel_trace.csv > $OUT/sequence.txt
rm -f $OUT/train_kernel_trace.csv
