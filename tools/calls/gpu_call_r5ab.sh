#!/bin/bash
# round 5 ab: full GPU suite + smoke + the bench line at HEAD (after the fused-epilogue, ConvT and band-kernel changes)
set -o pipefail
mkdir -p gpurun_out
export CDM_PARITY_OUT=gpurun_out/r5ab_parity.jsonl
rm -f $CDM_PARITY_OUT
timeout -k 10 800 python3 -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests/ > gpurun_out/r5ab_tests.log 2>&1
echo tests rc=$?
unset CDM_PARITY_OUT
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5ab_smoke.log 2>&1 || exit 1
echo smoke ok
timeout -k 10 500 python3 bench.py > gpurun_out/r5ab_bench.json 2> gpurun_out/r5ab_bench.err || exit 1
echo bench ok
