#!/bin/bash
# round 5 n: the N-rank bench path through bench.py's own launcher (--gpus 2), both ranks on the one GPU with gloo
# collectives (CDM_BENCH_REHEARSE=1; RCCL refuses two ranks on one device) — plumbing, not a scaling number
set -o pipefail
mkdir -p gpurun_out
CDM_BENCH_REHEARSE=1 timeout -k 10 600 python3 bench.py --gpus 2 --steps 5 --warmup 2 --sample-steps 10 --cfg-sample-steps 5 --no-extra --no-cpu > gpurun_out/r5n_rehearse.json 2> gpurun_out/r5n_rehearse.err
echo rehearse rc=$?
