"""Median-per-dispatch PMC values of the conv kernel from tools/pmc_x6.sh output dirs -> JSON on stdout."""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1]
out = {}
for f in sorted(glob.glob(os.path.join(root, "p*", "conv_counter_collection.csv"))):
    agg = collections.defaultdict(float)
    names = {}
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if ("gemm" not in k and "conv3x3" not in k) or "pack" in k:
            continue
        agg[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = k
    per = collections.defaultdict(list)
    for (d, c), v in agg.items():
        per[c].append(v)
    for c, v in per.items():
        v = sorted(v)
        out[c] = v[len(v) // 2]
    if names:
        out["kernel"] = sorted(set(names.values()))[0][:160]
if "SQ_VALU_MFMA_BUSY_CYCLES" in out and "GRBM_GUI_ACTIVE" in out:
    # GRBM_GUI_ACTIVE is summed over the 8 XCDs; MFMA busy over all 1024 SIMDs
    out["mfma_util"] = out["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / (out["GRBM_GUI_ACTIVE"] / 8)
if "FETCH_SIZE" in out and "WRITE_SIZE" in out:
    out["traffic_bytes"] = int(out["FETCH_SIZE"] * 1024 * 2 + out["WRITE_SIZE"] * 1024)
print(json.dumps(out, indent=1))
