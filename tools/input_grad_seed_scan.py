"""Seed scan for tests/test_gpu_input_grads.py: per input seed, the worst ratio of HIP's gradient error (vs fp64 autograd
of the oracle) to the reference's own fp32 error bar (3x + 2e-6), under fp32 / h3 and per-sample / broadcast t, c.  A
seed where every ratio is <= 1 has no ReLU / MaxPool kink that any arithmetic flips."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from oracle import ref_cpu as R  # noqa: E402
import test_gpu_input_grads as T  # noqa: E402


def run(seed, math, bcast):
    import cdm_amd
    torch.manual_seed(3 + 100 * seed)
    m = cdm_amd.ContextUnet(1, T.NF, T.NCF, T.H, conv_math=math).cuda().train()
    sd = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    g = torch.Generator().manual_seed(11 + 100 * seed)
    x = torch.randn(T.B, 1, T.H, T.H, generator=g)
    rows = 1 if bcast else T.B
    t = torch.rand(rows, generator=g); c = torch.rand(rows, T.NCF, generator=g)
    w = torch.randn(T.B, 1, T.H, T.H, generator=g)
    torch.manual_seed(21)
    sc = R.draw_shortcut(1, T.NF)
    xg, tg, cg = (v.cuda().requires_grad_(True) for v in (x, t, c))
    torch.manual_seed(21)
    (m(xg, tg, cg) * w.cuda()).sum().backward()
    _, dx64, dt64, dc64, g64 = T._oracle(sd, x, t, c, sc, torch.float64, w)
    _, dx32, dt32, dc32, g32 = T._oracle(sd, x, t, c, sc, torch.float32, w)
    worst = 0.0
    pairs = [(xg.grad.view(T.B, 1, T.H, T.H), dx64, dx32), (tg.grad, dt64, dt32), (cg.grad, dc64, dc32)]
    pairs += [(p.grad, g64[k], g32[k]) for k, p in m.named_parameters() if not k.endswith("0.bias") or "embed" in k]
    for h, r64, r32 in pairs:
        worst = max(worst, T._rel_l2(h, r64) / (3 * T._rel_l2(r32, r64) + 2e-6))
    return worst


if __name__ == "__main__":
    torch.set_num_threads(16)
    for seed in range(int(sys.argv[1]) if len(sys.argv) > 1 else 10):
        r = {f"{mth}/{'b' if b else 's'}": run(seed, mth, b) for mth in ("fp32", "h3") for b in (False, True)}
        print(seed, " ".join(f"{k} {v:.2f}" for k, v in r.items()), "OK" if max(r.values()) <= 1 else "", flush=True)
