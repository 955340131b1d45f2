#!/bin/bash
# A/B the train step / sampling under two environment settings, interleaved (same library):
#   bash tools/ab_env.sh "CDM_BN_SUMS=0" "CDM_BN_SUMS=1" [rounds]
set -e
A=$1; B=$2; N=${3:-2}
mkdir -p gpurun_out/ab
for r in $(seq 1 $N); do
  for E in "$A" "$B"; do
    n=$(echo "$E" | tr -c 'A-Za-z0-9_' '_')
    env $E timeout -k 10 300 python -u bench.py --no-cpu --no-extra --sample-steps 100 --cfg-sample-steps 20 > gpurun_out/ab/$n.$r.log 2>&1
    python - "$E" "gpurun_out/ab/$n.$r.log" <<'PY'
import json, sys
l = [x for x in open(sys.argv[2]) if x.startswith("{")][0]; d = json.loads(l)
print(sys.argv[1], "train_ms", d["ms_per_step"], "img/s", d["value"], "conv_ms", d["roofline"]["launch_ms"],
      "sample_ms", d["sample"]["ms_per_denoise_step"], "loss", d["final_loss"], flush=True)
PY
  done
done
