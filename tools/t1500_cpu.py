"""CPU-only control for the T=1500 nf=8 trajectory error: the reference loop in fp32 with
  (a) the oracle's fp32 eps   -> must reproduce the golden's fp32 final x (validates the RNG order of the loop),
  (b) the oracle's fp64 eps rounded to fp32, fp32 denoise  -> the error the fp32 denoise arithmetic alone leaves,
  (c) = (b) but the shortcut / x state handed to the fp64 forward as in the HIP probe (tools/t1500_steps.py),
and each final x's deviation from the golden fp64 trajectory.  No GPU.

    python tools/t1500_cpu.py [--w 0]
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import ref_cpu as R  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--w", type=float, default=0.0)
    ap.add_argument("--modes", default="fp32,fp64eps")
    a = ap.parse_args()
    torch.set_num_threads(8)
    g = os.path.join(ROOT, "tests", "golden")
    fx = np.load(os.path.join(g, "model_nf8.npz"))
    sd = {k[3:]: torch.from_numpy(fx[k].copy()) for k in fx.files if k.startswith("sd.")}
    sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}
    sfx = np.load(os.path.join(g, "sampler_T1500_nf8.npz"))
    T = int(sfx["T"]); nf, H, n = 8, 64, 2
    params = torch.from_numpy(sfx["params"])
    b32, a32, ab32 = R.make_schedule(T)
    ref64 = sfx[f"w{a.w:g}_x_fp64"]; ref32 = sfx[f"w{a.w:g}_x"]
    mx = np.abs(ref64).max()
    for mode in a.modes.split(","):
        t0 = time.time()
        torch.manual_seed(int(sfx[f"w{a.w:g}_seed"]))
        x = torch.randn(n, 1, H, H)
        for i in range(T, 0, -1):
            t = torch.tensor([i / T])
            z = torch.randn(n, 1, H, H) if i > 1 else 0
            conds = [params] + ([torch.zeros_like(params)] if a.w > 0 else [])
            outs = []
            for cc in conds:
                w_, b_ = R.draw_shortcut(1, nf)
                with torch.no_grad():
                    if mode == "fp32":
                        e = R.unet_forward(sd, x, t, cc, n_feat=nf, n_cfeat=6, height=H, train=False, shortcut=(w_, b_))
                    else:
                        e = R.unet_forward(sd64, x.double(), t.double(), cc.double(), n_feat=nf, n_cfeat=6, height=H,
                                           train=False, shortcut=(w_.double(), b_.double())).float()
                outs.append(e)
            eps = outs[0] if a.w == 0 else outs[1] + a.w * (outs[0] - outs[1])
            x = R.denoise_add_noise(x, i, eps, z, b32, a32, ab32)
        d = x.numpy() - ref64
        print(f"{mode}: final max|d|/max|x| {np.abs(d).max() / mx:.3e}  L2 rel {np.linalg.norm(d) / np.linalg.norm(ref64):.3e}"
              f"  bit-equal to golden fp32: {np.array_equal(x.numpy(), ref32)}  (max|x - golden32| "
              f"{np.abs(x.numpy() - ref32).max():.3g})  {time.time() - t0:.0f} s", flush=True)
        np.save(f"/tmp/t1500_cpu_{mode}.npy", x.numpy())


if __name__ == "__main__":
    main()
