#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export CDM_PARITY_OUT=gpurun_out/r5t_parity.jsonl
rm -f $CDM_PARITY_OUT
timeout -k 10 700 python3 -u -m pytest -v -s --timeout 400 --timeout-method thread -m gpu tests/test_gpu_trainer.py > gpurun_out/r5t_tests.log 2>&1
echo tests rc=$?
