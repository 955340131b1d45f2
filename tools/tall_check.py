"""A/B bit-exactness of a kernel-variant knob over whole train steps: runs the bench's seeded train step (graph-replayed)
for a few steps and writes every parameter (after the optimizer steps) to an npz; compare two runs made under two
environment settings:
  CDM_HALO_TALL=0 python tools/tall_check.py --out a.npz --math bf16
  CDM_HALO_TALL=1 python tools/tall_check.py --out b.npz --math bf16
  python tools/tall_check.py --cmp a.npz b.npz"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

ap = argparse.ArgumentParser()
ap.add_argument("--out")
ap.add_argument("--math", default="bf16")
ap.add_argument("--steps", type=int, default=3)
ap.add_argument("--cmp", nargs=2)
a = ap.parse_args()
if a.cmp:
    x, y = np.load(a.cmp[0]), np.load(a.cmp[1])
    bad = [k for k in x.files if not np.array_equal(x[k].view(np.uint32), y[k].view(np.uint32))]
    worst = max((float(np.abs(x[k] - y[k]).max()) for k in x.files), default=0.0)
    print(f"{len(x.files)} tensors, {len(bad)} differ (max |d| {worst:.3e})", bad[:8])
    sys.exit(0)
import torch  # noqa: E402

import bench  # noqa: E402

model, ms, loss = bench.train_rate(bench.NF, bench.H, bench.T, 256, a.math, a.steps, 0, 0, torch.cuda.synchronize)
np.savez(a.out, loss=np.array([loss], np.float32),
         **{k: v.detach().float().cpu().numpy() for k, v in model.state_dict().items() if v.is_floating_point()})
print(f"{a.math}: {ms:.3f} ms/step, loss {loss!r} -> {a.out}")
