"""Per-step kernel time by kernel family from a rocprofv3 kernel trace (steps delimited by adam_kernel).
    python tools/kstep.py gpurun_out/prof_train2/train_kernel_trace.csv [n_last_steps]"""
import collections
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
nl = int(sys.argv[2]) if len(sys.argv) > 2 else 10
idx = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
nl = min(nl, len(idx) - 1)
steps = [rows[idx[k] + 1: idx[k + 1] + 1] for k in range(len(idx) - 1 - nl, len(idx) - 1)]
agg = collections.Counter(); cnt = collections.Counter()
wall = 0.0
for st in steps:
    wall += (int(st[-1]["End_Timestamp"]) - int(st[0]["Start_Timestamp"])) / 1e3
    for r in st:
        n = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("cdm::", "")
        agg[n] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        cnt[n] += 1
ns = len(steps)
tot = sum(agg.values()) / ns
print(f"{ns} steps: kernel sum {tot / 1e3:.3f} ms/step, wall {wall / ns / 1e3:.3f} ms/step")
for n, v in agg.most_common():
    print(f"{v / ns:10.1f} us {cnt[n] // ns:4d}x {100 * v / ns / tot:5.1f}%  {n[:110]}")
