"""HBM traffic / MFMA counters of the roofline conv launches INSIDE the training step, from rocprofv3 --pmc CSVs.

The bench's dominant kernel is measured as the first 9 conv3x3_halo_x3_kernel<4, 64, ...> dispatches of each
training step (init_conv.conv2, down1 x4, up2 x4: the 128 -> 128 @64x64 forwards; steps delimited by adam_kernel;
the PreNone and PreBnRelu staging instances both count).  gfx950 corrections (MI355X_MICROARCH.md §HBM):
FETCH_SIZE is KiB and reads 1/2 of a wide coalesced read stream (x2); WRITE_SIZE is exact (KiB).

    python tools/pmc_step.py OUTDIR     (OUTDIR/p<i>/*counter_collection.csv from tools/pmc_step.sh)
"""
import collections
import csv
import glob
import json
import os
import statistics
import sys


def dispatches(path):
    rows = list(csv.DictReader(open(path)))
    by = collections.OrderedDict()
    for r in rows:
        d = int(r["Dispatch_Id"])
        e = by.setdefault(d, {"name": r["Kernel_Name"], "vals": {}})
        e["vals"][r["Counter_Name"]] = e["vals"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return [by[k] for k in sorted(by)]


# the roofline kernel's instantiation: h3 (4) by default, "conv3x3_halo_x3_kernel<1, 64," for the bf16 C4 step
KERNEL = os.environ.get("CDM_PMC_KERNEL", "conv3x3_halo_x3_kernel<4, 64,")
HALO_FETCH_PER_BYTE = 0.6706   # FETCH_SIZE per byte of the halo staging pattern (profiles/r3_fetch_calibration.txt)


def roofline_launches(ds):
    steps, cur = [], []
    for d in ds:
        if "adam_kernel" in d["name"]:
            steps.append(cur); cur = []
        else:
            cur.append(d)
    out = []
    for st in steps[2:]:                       # skip the warm-up / capture steps
        halo = [d for d in st if KERNEL in d["name"]]
        out.extend(halo[:9])
    return out


def main(outdir):
    vals = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(outdir, "p*", "**", "*counter_collection.csv"), recursive=True)):
        for d in roofline_launches(dispatches(f)):
            for k, v in d["vals"].items():
                vals[k].append(v)
    med = {k: statistics.median(v) for k, v in vals.items()}
    n = {k: len(v) for k, v in vals.items()}
    algo = 256 * 64 * 64 * 128 * 4 * 2 + 9 * 128 * 128 * 4 * 2 + 4096 * 2 * 128 * 4
    d = {"what": "per-launch medians over the roofline conv launches inside the training step", "launches": n,
         "median": med, "algorithmic_bytes": algo}
    if "FETCH_SIZE" in med and "WRITE_SIZE" in med:
        fb, wb = med["FETCH_SIZE"] * 1024 / HALO_FETCH_PER_BYTE, med["WRITE_SIZE"] * 1024
        d.update(fetch_bytes_corrected=fb, write_bytes=wb, traffic_bytes=fb + wb, traffic_over_algorithmic=(fb + wb) / algo)
    if "SQ_INSTS_MFMA" in med:
        d["mfma_insts"] = med["SQ_INSTS_MFMA"]
    d["note"] = ("FETCH_SIZE / 0.6706 (the halo staging pattern's calibrated counter rate, "
                 "profiles/r3_fetch_calibration.txt), KiB -> bytes; one counter group per rocprofv3 pass; "
                 "algorithmic = x read + y write + weights (fp16 hi/lo) + BN-stat partials")
    print(json.dumps(d, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
