#!/bin/bash
# round 5 f: eval-mode BN weight-gradient diagnostic with out.0's output gradient, then the in_channels tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/eval_dgamma_diag.py gpurun_out/r5f_eval_dgamma.npz > gpurun_out/r5f_diag.log 2>&1 || exit 1
echo diag ok
