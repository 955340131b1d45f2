"""Per-kernel A/B from tools/kstep.py breakdowns: mean per-launch time of every kernel under two settings, each run
one or more times on the same box (interleaved), and the per-step difference.

    python tools/kcmp.py A_dir1,A_dir2 B_dir1,B_dir2 [min_us]     (each dir holds breakdown.txt)
"""
import re
import sys


def load(path):
    out = {}
    for line in open(path):
        m = re.match(r"\s*([\d.]+) us\s+(\d+)x\s+[\d.]+%\s+(.+)$", line)
        if m:
            out[m.group(3).strip()] = (float(m.group(1)), int(m.group(2)))
    return out


def merged(dirs):
    runs = [load(d.rstrip("/") + "/breakdown.txt") for d in dirs.split(",")]
    keys = set().union(*runs)
    return {k: (sum(r.get(k, (0, 0))[0] for r in runs) / len(runs), max(r.get(k, (0, 0))[1] for r in runs))
            for k in keys}


a, b = merged(sys.argv[1]), merged(sys.argv[2])
floor = float(sys.argv[3]) if len(sys.argv) > 3 else 50.0
rows = []
for k in set(a) | set(b):
    ta, na = a.get(k, (0.0, 0))
    tb, nb = b.get(k, (0.0, 0))
    if max(ta, tb) < floor:
        continue
    n = max(na, nb)
    rows.append((tb - ta, k, ta, tb, n))
rows.sort()
print(f"{'d us/step':>10} {'A us/launch':>12} {'B us/launch':>12} {'n':>3}  kernel")
for d, k, ta, tb, n in rows:
    print(f"{d:10.1f} {ta / n:12.1f} {tb / n:12.1f} {n:3d}  {k[:150]}")
print(f"total A {sum(v[0] for v in a.values()):.1f} us/step, B {sum(v[0] for v in b.values()):.1f} us/step")
