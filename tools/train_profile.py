"""Train-step-only workload for kernel traces: the bench's C2 train step (bs=256, n_feat=128, hipGraph-replayed),
  rocprofv3 --kernel-trace --stats -- python3 tools/train_profile.py [--steps 20] [--math h3] [--no-graph]
Per-step kernel time = kernel_stats total / (warmup + steps)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--warmup", type=int, default=5)
ap.add_argument("--math", default="h3")
ap.add_argument("--no-graph", action="store_true")
ap.add_argument("--c5", action="store_true", help="BASELINE config 5: 256x256, n_feat=256, T=2000, bs=16")
a = ap.parse_args()
nf, H, T, B = (256, 256, 2000, 16) if a.c5 else (bench.NF, bench.H, bench.T, 256)
_, ms, loss = bench.train_rate(nf, H, T, B, a.math, a.steps, a.warmup, 0,
                               torch.cuda.synchronize, use_graph=not a.no_graph)
print(f"train {ms:.3f} ms/step = {B / ms * 1e3:.1f} img/s (math {a.math}, {a.warmup}+{a.steps} steps), loss {loss:.5f}")
