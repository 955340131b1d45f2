#!/bin/bash
# Round profile collection on the GPU box (run through gpurun from the repo root).
#   1) kernel trace + stats of the bench command (sampling shortened to 100 of the 1500 steps)
#   2) two PMC passes on the dominant conv alone (shipped path): FETCH_SIZE, then WRITE_SIZE
set -e
OUT=${1:-gpurun_out/prof}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- \
    python3 bench.py --steps 20 --warmup 5 --sample-steps 100 --no-cpu > $OUT/bench_under_rocprof.json 2> $OUT/trace.err
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o conv -- python3 tools/conv_only.py 10 > /dev/null 2> $OUT/pmc_fetch.err
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o conv -- python3 tools/conv_only.py 10 > /dev/null 2> $OUT/pmc_write.err
rm -f $OUT/trace/bench_kernel_trace.csv
ls -la $OUT/trace $OUT/pmc_fetch $OUT/pmc_write
