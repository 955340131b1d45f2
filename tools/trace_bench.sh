#!/bin/bash
# Kernel trace + stats of a short bench run (no PMC): bash tools/trace_bench.sh <outdir> [bench args...]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/${1:-gpurun_out/trace}
shift || true
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o bench -- \
    python3 $R/bench.py --steps 10 --warmup 3 --sample-steps 50 --cfg-sample-steps 10 --no-cpu --no-extra "$@" \
    > $OUT/bench.json 2> $OUT/trace.err
rm -f $OUT/bench_kernel_trace.csv
python3 $R/tools/kstats.py $OUT/bench_kernel_stats.csv > $OUT/summary.txt
