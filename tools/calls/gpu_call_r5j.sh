#!/bin/bash
# round 5 j: ConvT weight gradient on the transposed-read staging — kernel / e2e tests, then a same-box A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_c2_e2e.py tests/test_gpu_c4_e2e.py tests/test_gpu_configs.py > gpurun_out/r5j_tests.log 2>&1 || exit 1
echo tests ok
for v in 0 1 0 1; do
  CDM_CONVT_WGRAD_TR=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --sample-steps 10 --cfg-sample-steps 0 --extra-sample-steps 10 --no-cpu > gpurun_out/r5j_ab_$v.json 2>> gpurun_out/r5j_ab.err || exit 1
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r5j_ab_$v.json').read().strip().splitlines()[-1]); print('tr=$v', d['ms_per_step'], d['configs']['c4_bf16_cfg']['train_ms_per_step'])" >> gpurun_out/r5j_ab.txt
done
echo ab ok
