#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 180 python3 -u tools/apply_probe.py > gpurun_out/r5i_apply.json 2> gpurun_out/r5i_apply.err || exit 1
echo probe ok
timeout -k 10 400 python3 -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_in_channels.py tests/test_gpu_blocks.py > gpurun_out/r5i_tests.log 2>&1 || exit 1
echo tests ok
