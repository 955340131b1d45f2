"""Summarise hipcc -Rpass-analysis=kernel-resource-usage remarks (stdin or a file): one line per kernel with
VGPRs / AGPRs / spills / scratch / occupancy / LDS, demangled, optionally filtered by a substring.

    hipcc ... -Rpass-analysis=kernel-resource-usage -c csrc/gemm_f32.hip -o /tmp/g.o 2> /tmp/ru.txt
    python tools/res_usage.py /tmp/ru.txt halo wgrad
"""
import re
import subprocess
import sys

txt = open(sys.argv[1]).read()
filters = sys.argv[2:]
rows, cur = [], None
for line in txt.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+([A-Za-z \[\]/]+?):\s+(\d+)", line)
    if m and cur is not None:
        cur[m.group(1).strip()] = int(m.group(2))
names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True,
                       text=True).stdout.splitlines()
for r, n in zip(rows, names):
    if filters and not any(f in n for f in filters):
        continue
    print(f"V{r.get('VGPRs', 0):4d} A{r.get('AGPRs', 0):4d} spill{r.get('VGPRs Spill', 0):4d} "
          f"scr{r.get('ScratchSize [bytes/lane]', 0):4d} occ{r.get('Occupancy [waves/SIMD]', 0)} "
          f"lds{r.get('LDS Size [bytes/block]', 0):7d}  {n[:170]}")
