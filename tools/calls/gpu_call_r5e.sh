#!/bin/bash
# round 5 e: smoke, the round's rocprof kernel summary + PMC of the dominant conv, then the full bench line
set -o pipefail
mkdir -p gpurun_out
export CDM_PARITY_OUT=gpurun_out/r5e_parity.jsonl
timeout -k 10 400 python3 -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_input_grads.py > gpurun_out/r5e_tests.log 2>&1 || exit 1
echo tests ok
unset CDM_PARITY_OUT
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5e_smoke.log 2>&1 || exit 1
echo smoke ok
timeout -k 10 1000 bash tools/gpu_profile.sh gpurun_out/r5_prof h3 > gpurun_out/r5e_prof.log 2>&1 || exit 1
echo profile ok
timeout -k 10 600 python3 bench.py > gpurun_out/r5e_bench.json 2> gpurun_out/r5e_bench.err || exit 1
echo bench ok
