"""Summarise a rocprofv3 kernel trace of tools/rccl_trace.py: the last training step's kernels in start order with their
times relative to the step start, the collective (RCCL / NCCL) kernels marked, and how much backward work ran after
each collective was enqueued (the overlap the stage-bucketed all-reduce allows).

    python tools/rccl_timeline.py gpurun_out/r3_rccl/rccl_kernel_trace.csv > profiles/r3_rccl_timeline.txt
"""
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
adam = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
if len(adam) < 2:
    sys.exit("fewer than two steps in the trace")
step = rows[adam[-2] + 1: adam[-1] + 1]
t0 = int(step[0]["Start_Timestamp"])
t_end = int(step[-1]["End_Timestamp"])
is_coll = lambda n: bool(re.search(r"nccl|rccl|AllReduce|allreduce", n, re.I))  # noqa: E731
print(f"last step: {len(step)} kernels, {(t_end - t0) / 1e3:.1f} us from first start to Adam end")
ncoll = 0
for r in step:
    n = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("cdm::", "")
    s = (int(r["Start_Timestamp"]) - t0) / 1e3
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    mark = ""
    if is_coll(r["Kernel_Name"]):
        ncoll += 1
        after = sum(1 for q in step if int(q["Start_Timestamp"]) > int(r["Start_Timestamp"])
                    and not is_coll(q["Kernel_Name"]) and "adam" not in q["Kernel_Name"])
        mark = f"   <== collective #{ncoll}: {after} backward kernels start after it"
    print(f"{s:10.1f} us  {d:8.1f} us  {n[:90]}{mark}")
print(f"collective kernels in the step: {ncoll}")
