#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_in_channels.py > gpurun_out/r5o_tests.log 2>&1
echo tests rc=$?
