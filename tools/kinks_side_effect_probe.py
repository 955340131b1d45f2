"""Does reading HIP's decisions (tests/_kinks.py::hip_kinks, one extra engine forward) before a Trainer step change
that step?  Two identical 3-step Trainer runs (h3, n_feat 8, seed 0 of test_trainer_three_steps_all_arithmetics), one
with hip_kinks before every step: the step gradients must be bit-identical (GPU box).

    python tools/kinks_side_effect_probe.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]


def run(with_kinks, math="h3", seed=0, nf=8, B=4, T=1000, lrs=(1e-3, 1e-3, 7.5e-4)):
    import cdm_amd
    from cdm_amd import Trainer
    from oracle import ref_cpu as R
    from _kinks import hip_kinks
    torch.manual_seed(100 + seed)
    m = cdm_amd.ContextUnet(1, nf, 6, 64, conv_math=math).cuda().train()
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(B, 1, 64, 64, generator=g); c = torch.rand(B, 6, generator=g)
    draws = [(torch.randn(B, 1, 64, 64, generator=g), torch.randint(1, T + 1, (B,), generator=g),
              torch.rand(2 * nf, generator=g) * 2 - 1) for _ in lrs]
    tr = Trainer(m, lrs[0], T, B, use_graph=False)
    _, _, ab = R.make_schedule(T)
    out = []
    for lr, (noise, t, sc) in zip(lrs, draws):
        if with_kinks:
            state = {kk: v.detach().clone() for kk, v in m.state_dict().items()}
            xp = R.perturb_input(x, t, noise, ab)
            hip_kinks(m, xp, t / T, c, (sc[:nf].reshape(nf, 1, 1, 1), sc[nf:]), frozen=False)
            m.load_state_dict(state)
        tr.set_lr(lr)
        tr.step(x.cuda(), c.cuda(), inject=(noise.cuda(), t.cuda().int(), sc.cuda()))
        torch.cuda.synchronize()
        out.append({n: v.detach().cpu().clone() for n, v in tr.grads.items()})
    return out


def main():
    a, b = run(False), run(True)
    for k, (ga, gb) in enumerate(zip(a, b)):
        diff = [n for n in ga if not torch.equal(ga[n], gb[n])]
        print(f"step {k}: {len(diff)} of {len(ga)} gradient tensors differ", diff[:6])


if __name__ == "__main__":
    main()
