#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python3 -u tools/mfma_round_probe.py > gpurun_out/r5g_mfma_round.json 2> gpurun_out/r5g_mfma_round.err || exit 1
echo probe ok
