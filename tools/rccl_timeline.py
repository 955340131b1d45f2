"""Summarise a rocprofv3 trace of tools/rccl_trace.py (the Trainer's data-parallel path over RCCL).

    rocprofv3 --kernel-trace --rccl-trace --hip-runtime-trace --output-format csv -d gpurun_out/r3_rccl -o rccl \
        -- python3 tools/rccl_trace.py
    python tools/rccl_timeline.py gpurun_out/r3_rccl > profiles/r3_rccl_timeline.txt

Part 1, host order of the last training step: every kernel launch (hipLaunchKernel / hipModuleLaunchKernel / graph
launch, named through its correlation id in the kernel trace) and every RCCL API call, so one sees each stage's
all-reduce being enqueued as soon as that stage's last gradient kernel is launched, with the rest of the backward
launched after it.  Part 2, GPU order: the step's kernels with device times; collective kernels are marked (a one-rank
group runs none: RCCL completes a single-rank all-reduce without a device kernel).
"""
import csv
import glob
import os
import re
import sys


def load(d, suffix):
    f = glob.glob(os.path.join(d, f"*{suffix}"))
    return list(csv.DictReader(open(f[0]))) if f else []


def short(n):
    return re.sub(r"\(.*", "", n).replace("void ", "").replace("cdm::", "")[:80]


d = sys.argv[1]
kern = sorted(load(d, "kernel_trace.csv"), key=lambda r: int(r["Start_Timestamp"]))
hip = load(d, "hip_api_trace.csv")
rccl = load(d, "rccl_api_trace.csv")
name_of = {r["Correlation_Id"]: short(r["Kernel_Name"]) for r in kern}
adam_k = [i for i, r in enumerate(kern) if "adam_kernel" in r["Kernel_Name"]]
if len(adam_k) < 2:
    sys.exit("fewer than two steps in the kernel trace")

# ---- part 1: host order ----
ev = []
for r in hip:
    if "Launch" in r["Function"] and r["Correlation_Id"] in name_of:
        ev.append((int(r["Start_Timestamp"]), "launch", name_of[r["Correlation_Id"]]))
for r in rccl:
    ev.append((int(r["Start_Timestamp"]), "rccl", r["Function"]))
ev.sort()
adam_h = [i for i, e in enumerate(ev) if e[1] == "launch" and "adam_kernel" in e[2]]
print(f"RCCL API calls in the trace: {len(rccl)}; kernel launches traced: {sum(1 for e in ev if e[1] == 'launch')}")
if len(adam_h) >= 2:
    step = ev[adam_h[-2] + 1: adam_h[-1] + 1]
    t0 = step[0][0]
    nl = sum(1 for e in step if e[1] == "launch")
    print(f"\n== part 1: host order of the last step ({nl} kernel launches) ==")
    for k, (t, kind, n) in enumerate(step):
        if kind == "rccl":
            after = sum(1 for e in step[k + 1:] if e[1] == "launch" and "adam" not in e[2])
            print(f"{(t - t0) / 1e3:10.1f} us  RCCL {n}   <== {after} backward kernel launches follow it")
        else:
            print(f"{(t - t0) / 1e3:10.1f} us  launch {n}")
else:
    print("(no HIP API trace: part 1 skipped)")

# ---- part 2: GPU order ----
step = kern[adam_k[-2] + 1: adam_k[-1] + 1]
t0 = int(step[0]["Start_Timestamp"])
is_coll = lambda n: bool(re.search(r"nccl|rccl|AllReduce|allreduce", n, re.I))  # noqa: E731
ncoll = sum(1 for r in step if is_coll(r["Kernel_Name"]))
print(f"\n== part 2: device order of the last step: {len(step)} kernels, "
      f"{(int(step[-1]['End_Timestamp']) - t0) / 1e3:.1f} us from first start to Adam end; collective kernels: {ncoll} ==")
for r in step:
    s = (int(r["Start_Timestamp"]) - t0) / 1e3
    du = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    print(f"{s:10.1f} us  {du:8.1f} us  {short(r['Kernel_Name'])}{'   <== collective' if is_coll(r['Kernel_Name']) else ''}")
