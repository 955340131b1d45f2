#!/bin/bash
# Round profile collection on the GPU box (run through gpurun from the repo root).
#   1) kernel trace + stats of the bench command (sampling shortened to 100 of the 1500 steps, CFG legs 20 steps:
#      round 5's run under rocprofv3 aborted its queue at the first CFG graph replay, HSA_STATUS_ERROR_INVALID_PACKET_
#      FORMAT; round 6's profiled run with the CFG legs on completed, tools/calls/r6a.sh, and the CFG path's fused
#      epilogue is now checked at the bench's 512-image batch, tests/test_gpu_sample_bench_shape.py)
#   2) PMC passes on the dominant conv alone in the shipped arithmetic (tools/pmc_x6.sh: one counter
#      group per pass, incl. FETCH_SIZE and WRITE_SIZE in separate passes)
#   bash tools/gpu_profile.sh [outdir] [conv_math]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/${1:-gpurun_out/prof}
MODE=${2:-x6}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- \
    python3 $R/bench.py --steps 20 --warmup 5 --sample-steps 100 --cfg-sample-steps 20 --no-cpu --no-extra --conv-math $MODE \
    > $OUT/bench_under_rocprof.json 2> $OUT/trace.err
rm -f $OUT/trace/bench_kernel_trace.csv
timeout -k 10 900 bash $R/tools/pmc_x6.sh $MODE ${1:-gpurun_out/prof}/pmc > /dev/null
ls -la $OUT/trace $OUT/pmc
