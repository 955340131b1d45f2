#!/bin/bash
# A/B the C5 train step (256x256, n_feat=256, bs=16) of two library builds, interleaved:  bash tools/ab_c5.sh A.so B.so [rounds]
set -e
A=$1; B=$2; N=${3:-2}
for r in $(seq 1 $N); do
  for L in $A $B; do
    echo -n "$(basename $L .so) "
    CDM_LIB=$L timeout -k 10 300 python -u tools/train_profile.py --c5 --steps 4 --warmup 2
  done
done
