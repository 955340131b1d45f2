#!/bin/bash
# round 5 l: rocprof kernel summary + PMC of the dominant conv at HEAD, then the full bench line
set -o pipefail
mkdir -p gpurun_out
rm -rf gpurun_out/r5_prof
timeout -k 10 1000 bash tools/gpu_profile.sh gpurun_out/r5_prof h3 > gpurun_out/r5l_prof.log 2>&1 || exit 1
echo profile ok
timeout -k 10 600 python3 bench.py > gpurun_out/r5l_bench.json 2> gpurun_out/r5l_bench.err || exit 1
echo bench ok
