"""The launch sequence of one training step (the last full one: between the last two adam_kernel dispatches) from a
rocprofv3 kernel trace, with each launch's duration and grid — to map kernel families to layers.
    python tools/kseq.py trace.csv [step_from_end]"""
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
back = int(sys.argv[2]) if len(sys.argv) > 2 else 1
idx = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
a, b = idx[-1 - back], idx[-back]
for k, r in enumerate(rows[a + 1: b + 1]):
    n = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("cdm::", "")
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    grid = "x".join(r.get(f"Grid_Size_{c}", r.get(f"Grid_{c}", "?")) for c in "XYZ")
    print(f"{k:4d} {d:9.1f} us  grid {grid:>16s}  {n[:150]}")
