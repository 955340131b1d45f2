"""Per-kernel-family PMC medians inside the training step, from rocprofv3 --pmc CSVs (tools/pmc_step.sh passes).
Kernel names are grouped by their template text; steps are delimited by adam_kernel and the first 2 skipped.
FETCH_SIZE is reported x2 (gfx950 wide-read correction, MI355X_MICROARCH.md §HBM), KiB -> bytes.
    python tools/pmc_families.py OUTDIR [name-substring ...]"""
import collections
import csv
import glob
import json
import os
import re
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_step import dispatches  # noqa: E402


def main(outdir, subs):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(outdir, "p*", "**", "*counter_collection.csv"), recursive=True)):
        steps, cur = [], []
        for d in dispatches(f):
            if "adam_kernel" in d["name"]:
                steps.append(cur); cur = []
            else:
                cur.append(d)
        for st in steps[2:]:
            for d in st:
                n = re.sub(r"\(.*", "", d["name"]).replace("void ", "").replace("cdm::", "")
                if subs and not any(s in n for s in subs):
                    continue
                for k, v in d["vals"].items():
                    vals[n][k].append(v)
    out = {}
    for n, kv in vals.items():
        med = {k: statistics.median(v) for k, v in kv.items()}
        if "FETCH_SIZE" in med:
            med["fetch_bytes_x2"] = med["FETCH_SIZE"] * 2048
            if "halo" in n:   # the halo staging pattern's calibrated counter rate (profiles/r3_fetch_calibration.txt)
                med["fetch_bytes_halo_cal"] = med["FETCH_SIZE"] * 1024 / 0.6706
        if "WRITE_SIZE" in med:
            med["write_bytes"] = med["WRITE_SIZE"] * 1024
        w = med.get("SQ_WAVE_CYCLES")
        if w:
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if k in med:
                    med[k + "_frac"] = med[k] / w
        if "SQ_INSTS_MFMA" in med and "GRBM_GUI_ACTIVE" in med:
            med["mfma_busy_frac"] = med["SQ_INSTS_MFMA"] * 32 / 1024 / (med["GRBM_GUI_ACTIVE"] / 8)
        out[n] = {k: round(v, 4) if isinstance(v, float) else v for k, v in med.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
