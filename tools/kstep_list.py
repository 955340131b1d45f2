"""Per-launch list of one reverse-diffusion step from a rocprofv3 kernel trace (the second-to-last complete step):
    python tools/kstep_list.py trace.csv [delimiter]"""
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
delim = sys.argv[2] if len(sys.argv) > 2 else "denoise_kernel"
idx = [i for i, r in enumerate(rows) if delim in r["Kernel_Name"]]
for r in rows[idx[-3] + 1: idx[-2] + 1]:
    n = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("cdm::", "")
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    print(f"{d:9.1f} us grid {r.get('Grid_Size_X', r.get('Grid_Size', ''))} wg "
          f"{r.get('Workgroup_Size_X', r.get('Workgroup_Size', ''))} {n[:120]}")
