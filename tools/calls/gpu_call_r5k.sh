#!/bin/bash
# round 5 k: the full GPU suite at HEAD (parity records) and smoke
set -o pipefail
mkdir -p gpurun_out
export CDM_PARITY_OUT=gpurun_out/r5k_parity.jsonl
rm -f $CDM_PARITY_OUT
timeout -k 10 1000 python3 -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests/ > gpurun_out/r5k_tests.log 2>&1
echo tests rc=$?
unset CDM_PARITY_OUT
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5k_smoke.log 2>&1
echo smoke rc=$?
