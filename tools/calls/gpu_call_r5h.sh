#!/bin/bash
# round 5 h: the round's rocprof kernel summary (no CFG legs under the profiler) + PMC of the dominant conv, then the
# full bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 bash tools/gpu_profile.sh gpurun_out/r5_prof h3 > gpurun_out/r5h_prof.log 2>&1 || exit 1
echo profile ok
timeout -k 10 600 python3 bench.py > gpurun_out/r5h_bench.json 2> gpurun_out/r5h_bench.err || exit 1
echo bench ok
