#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/kinks_side_effect_probe.py > gpurun_out/r5u_probe.log 2>&1
echo probe rc=$?
