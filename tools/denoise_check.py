"""denoise_add_noise (code/train_diffusion_condition.py:274-279) on the HIP kernel vs the CPU oracle at EVERY step
index of T = 1500 and at trajectory magnitudes (|x| up to 1e4): count of elements that differ, per i range.

    python tools/denoise_check.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import ref_cpu as R  # noqa: E402


def main():
    import cdm_amd
    T = 1500
    sched = cdm_amd.Schedule(T, "cuda")
    b, a, ab = R.make_schedule(T)
    g = torch.Generator().manual_seed(1)
    n = 1 << 16
    bad_total = 0
    for scale in (1.0, 1e2, 1e4):
        x = torch.randn(n, generator=g) * scale
        eps = torch.randn(n, generator=g)
        z = torch.randn(n, generator=g)
        xd, ed, zd = x.cuda(), eps.cuda(), z.cuda()
        bad_i = []
        for i in range(T, 0, -1):
            ref = R.denoise_add_noise(x, i, eps, z if i > 1 else 0, b, a, ab)
            got = cdm_amd.denoise_add_noise(xd, i, ed, zd if i > 1 else 0, sched).cpu()
            nb = int((got != ref).sum())
            if nb:
                bad_i.append((i, nb, float((got - ref).abs().max() / ref.abs().max())))
        bad_total += len(bad_i)
        print(f"scale {scale:g}: {len(bad_i)} of {T} steps differ; first {bad_i[:8]}", flush=True)
    # the coefficient tables themselves vs the reference's scalar expressions
    coef = sched.coef.cpu(); sa = sched.sa.cpu(); sb = sched.sb.cpu()
    dc = sum(int(coef[i] != ((1 - a[i]) / (1 - ab[i]).sqrt())) for i in range(1, T + 1))
    da = sum(int(sa[i] != a[i].sqrt()) for i in range(1, T + 1))
    db = sum(int(sb[i] != b.sqrt()[i]) for i in range(1, T + 1))
    print(f"table entries differing from the reference's scalar expressions: coef {dc}, sqrt(a) {da}, sqrt(b) {db}")


if __name__ == "__main__":
    main()
