#!/bin/bash
# round 5 d: eval-mode BN weight-gradient diagnostic, then the full GPU suite at HEAD with parity records
set -o pipefail
mkdir -p gpurun_out
export CDM_PARITY_OUT=gpurun_out/r5d_parity.jsonl
timeout -k 10 300 python3 -u tools/eval_dgamma_diag.py gpurun_out/r5d_eval_dgamma.npz > gpurun_out/r5d_diag.log 2>&1 || exit 1
echo diag rc=$?
timeout -k 10 1000 python3 -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests/ > gpurun_out/r5d_tests.log 2>&1
echo tests rc=$?
