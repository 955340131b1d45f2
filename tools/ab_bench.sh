#!/bin/bash
# A/B the train step / sampling of two library builds on one box, interleaved:  bash tools/ab_bench.sh A.so B.so [rounds]
set -e
A=$1; B=$2; N=${3:-2}
mkdir -p gpurun_out/ab
for r in $(seq 1 $N); do
  for L in $A $B; do
    n=$(basename $L .so)
    CDM_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu --no-extra --sample-steps 100 --cfg-sample-steps 20 > gpurun_out/ab/$n.$r.log 2>&1
    python - "$n" "gpurun_out/ab/$n.$r.log" <<'PY'
import json, sys
l = [x for x in open(sys.argv[2]) if x.startswith("{")][0]; d = json.loads(l)
print(sys.argv[1], "train_ms", d["ms_per_step"], "img/s", d["value"], "conv_ms", d["roofline"]["launch_ms"],
      "sample_ms", d["sample"]["ms_per_denoise_step"], "cfg_ms", d["sample"]["cfg"]["w=1"]["ms_per_denoise_step"], flush=True)
PY
  done
done
