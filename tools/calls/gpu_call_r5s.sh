#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export CDM_PARITY_OUT=gpurun_out/r5s_parity.jsonl
rm -f $CDM_PARITY_OUT
timeout -k 10 600 python3 -u -m pytest -v -s --timeout 400 --timeout-method thread -m gpu tests/test_gpu_sampler.py -k "nf128_T1500 or host" > gpurun_out/r5s_tests.log 2>&1
echo tests rc=$?
