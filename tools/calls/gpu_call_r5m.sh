#!/bin/bash
# round 5 m: C4 tests incl. the nf128 T=1500 bf16 trajectory (emulation now rounds up0 too)
set -o pipefail
mkdir -p gpurun_out
export CDM_PARITY_OUT=gpurun_out/r5m_parity.jsonl
rm -f $CDM_PARITY_OUT
timeout -k 10 900 python3 -u -m pytest -v -s --timeout 400 --timeout-method thread -m gpu tests/test_gpu_configs.py tests/test_gpu_c4_e2e.py > gpurun_out/r5m_tests.log 2>&1
echo tests rc=$?
