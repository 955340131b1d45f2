#!/bin/bash
# round 5 p: BN-backward dy pass with hoisted coefficients — kernel test, then C4 same-box A/B of CDM_DY_PASS
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "bn_bwd_dy" > gpurun_out/r5p_tests.log 2>&1 || exit 1
echo tests ok
rm -f gpurun_out/r5p_ab.txt
for v in 0 1 0 1; do
  CDM_DY_PASS=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --sample-steps 10 --cfg-sample-steps 0 --extra-sample-steps 10 --no-cpu > gpurun_out/r5p_ab_$v.json 2>> gpurun_out/r5p_ab.err || exit 1
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r5p_ab_$v.json').read().strip().splitlines()[-1]); print('dy_pass=$v', d['ms_per_step'], d['configs']['c4_bf16_cfg']['train_ms_per_step'])" >> gpurun_out/r5p_ab.txt
done
echo ab ok
