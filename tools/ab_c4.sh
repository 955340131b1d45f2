#!/bin/bash
# A/B the C4 (bf16) and C2 (h3) train steps under two environment settings, interleaved (same library):
#   bash tools/ab_c4.sh "CDM_X=0" "CDM_X=1" [rounds]
set -e
A=$1; B=$2; N=${3:-2}
for r in $(seq 1 $N); do
  for E in "$A" "$B"; do
    for M in bf16 h3; do
      echo -n "$E $M: "
      env $E timeout -k 10 200 python -u tools/train_profile.py --math $M --steps 20 --warmup 5 2>/dev/null | tail -1
    done
  done
done
