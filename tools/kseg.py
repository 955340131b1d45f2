"""Per-segment kernel time by kernel family from a rocprofv3 kernel trace: segments end at each dispatch of the
delimiter kernel (default denoise_kernel: one reverse-diffusion step).
    python tools/kseg.py trace.csv [delimiter] [n_last_segments]"""
import collections
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
delim = sys.argv[2] if len(sys.argv) > 2 else "denoise_kernel"
nl = int(sys.argv[3]) if len(sys.argv) > 3 else 10
idx = [i for i, r in enumerate(rows) if delim in r["Kernel_Name"]]
segs = [rows[idx[k] + 1: idx[k + 1] + 1] for k in range(max(0, len(idx) - 1 - nl), len(idx) - 1)]
agg = collections.Counter(); cnt = collections.Counter()
wall = 0.0
for st in segs:
    wall += (int(st[-1]["End_Timestamp"]) - int(st[0]["Start_Timestamp"])) / 1e3
    for r in st:
        n = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("cdm::", "")
        agg[n] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        cnt[n] += 1
ns = len(segs)
tot = sum(agg.values()) / ns
print(f"{ns} segments: kernel sum {tot / 1e3:.3f} ms, wall {wall / ns / 1e3:.3f} ms")
for n, v in agg.most_common():
    print(f"{v / ns:10.1f} us {cnt[n] // ns:4d}x {100 * v / ns / tot:5.1f}%  {n[:110]}")
