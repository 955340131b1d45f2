"""Sampling-only workload for kernel traces: the bench's C2 reverse-diffusion step (n=256, T=1500, hipGraph-replayed),
  rocprofv3 --kernel-trace --stats -- python3 tools/sample_profile.py [--steps 60] [--w 0]
Per-step kernel time = kernel_stats total / steps (the capture's own launches aside)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=60)
ap.add_argument("--w", type=float, default=0.0)
ap.add_argument("--n", type=int, default=256)
ap.add_argument("--math", default="h3")
a = ap.parse_args()
import cdm_amd  # noqa: E402
torch.manual_seed(0)
model = cdm_amd.ContextUnet(1, bench.NF, bench.NCF, bench.H, conv_math=a.math).cuda().eval()
ms, S = bench.sample_rate(model, bench.T, a.n, a.w, a.steps, 0, torch.cuda.synchronize)
print(f"sample {ms:.3f} ms per denoise step (n={a.n}, w={a.w:g}, {S} steps)")
