"""Mean per dispatch of every counter in rocprofv3 counter_collection.csv files (one table per file).
    python tools/pmc_sum.py gpurun_out/pmc_halo/p*/..._counter_collection.csv"""
import collections
import csv
import glob
import sys

for pat in sys.argv[1:]:
    for f in sorted(glob.glob(pat, recursive=True)):
        agg = collections.defaultdict(float); disp = collections.defaultdict(set)
        for r in csv.DictReader(open(f)):
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            disp[r["Counter_Name"]].add(r["Dispatch_Id"])
        print(f)
        for k in sorted(agg):
            print(f"  {k:32s} {agg[k] / max(1, len(disp[k])):16.4g}  ({len(disp[k])} dispatches)")
