#!/bin/bash
# A/B the C4 (bf16) and C2 (h3) train steps of two library builds, interleaved:  bash tools/ab_lib.sh A.so B.so [rounds]
set -e
A=$1; B=$2; N=${3:-2}
for r in $(seq 1 $N); do
  for L in $A $B; do
    for M in bf16 h3; do
      echo -n "$(basename $L .so) $M: "
      CDM_LIB=$L timeout -k 10 200 python -u tools/train_profile.py --math $M --steps 20 --warmup 5 2>/dev/null | tail -1
    done
  done
done
