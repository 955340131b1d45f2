"""Fold rocprofv3 PMC CSVs (FETCH_SIZE / WRITE_SIZE passes on tools/conv_only.py) into per-launch HBM bytes.

gfx950 corrections (MI355X_MICROARCH.md §HBM): counters are KiB; FETCH_SIZE reads exactly 1/2 of the bytes of a
wide (16 B/lane) coalesced read stream -> x2; WRITE_SIZE is exact for 16-B stores.

    python tools/pmc_to_json.py FETCH.csv WRITE.csv OUT.json
"""
import csv
import json
import statistics
import sys


def med(path, key="gemm_f32_kernel"):
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open(path)) if key in r["Kernel_Name"]]
    return statistics.median(v), len(v), next(r["Kernel_Name"] for r in csv.DictReader(open(path)) if key in r["Kernel_Name"])


def main(fetch, write, out):
    f, nf, name = med(fetch)
    w, nw, _ = med(write)
    fb, wb = f * 1024 * 2, w * 1024
    algo = 256 * 64 * 64 * 128 * 4 * 2 + 9 * 128 * 128 * 4 + 8192 * 2 * 128 * 4
    d = {"kernel": name.split("(")[0], "launches": [nf, nw], "fetch_size_kib_median": f, "write_size_kib_median": w,
         "fetch_bytes_corrected": fb, "write_bytes": wb, "traffic_bytes": fb + wb,
         "algorithmic_bytes": algo, "traffic_over_algorithmic": (fb + wb) / algo,
         "note": "FETCH_SIZE x2 (gfx950 wide-read correction), KiB->bytes; medians over launches; separate passes"}
    json.dump(d, open(out, "w"), indent=1)
    print(json.dumps(d, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
