"""oracle.adam_step_restated (the arithmetic cdm_adam implements) pinned to torch.optim.Adam on this host — the
build container, where the reference's own training golden vectors (tests/golden/train_nf8.npz) were produced.

torch's CPU Adam here (torch 2.10, AVX-512 kernels): lerp_ and the addcmul_ are fused multiply-adds, addcdiv_ is
self + (value * t1) / t2, and sqrt goes through a vectorised math library that is not always correctly rounded.
The restatement uses a correctly rounded sqrt, so a small fraction of parameters may differ by an ulp-level amount;
exp_avg / exp_avg_sq (no sqrt) must match bit for bit."""
import numpy as np
import pytest
import torch

from oracle import ref_cpu as R


@pytest.mark.parametrize("n", [1_000_003, 37, 4096])
def test_restated_adam_matches_torch_adam(n):
    g = torch.Generator().manual_seed(n)
    p0 = torch.randn(n, generator=g)
    tp = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([tp], lr=1e-3)
    p, m, v = p0.numpy().copy(), np.zeros(n, np.float32), np.zeros(n, np.float32)
    for step, lr in enumerate((1e-3, 1e-3, 7.5e-4, 7.5e-4, 3e-4, 3e-4), start=1):
        grad = torch.randn(n, generator=g) * 10.0 ** (step - 3)
        opt.param_groups[0]["lr"] = lr
        tp.grad = grad.clone()
        opt.step()
        pre = p
        p, m, v = R.adam_step_restated(p, grad.numpy(), m, v, lr, step)
        st = opt.state[tp]
        assert np.array_equal(st["exp_avg"].numpy(), m)
        assert np.array_equal(st["exp_avg_sq"].numpy(), v)
        ref = tp.detach().numpy()
        frac = float((p == ref).mean())
        err = np.abs(p.astype(np.float64) - ref)
        assert (err <= np.spacing(np.abs(ref)) + np.abs(ref.astype(np.float64) - pre) * 2.0 ** -18).all()
        assert frac >= 0.999, frac
        p = ref.copy()                       # continue from torch's parameters (m / v are identical)


def test_restated_adam_bias_table_matches_device_table():
    """The trainer's device table holds exactly the Python-float bias corrections the restatement (and torch) use."""
    import sys, os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from cdm_amd.trainer import adam_bias_table
    t = adam_bias_table(0.9, 0.999).numpy()
    for s in (1, 2, 3, 10, 100, 1000, 40000, 40960):
        assert t[s - 1, 0] == 1 - 0.9 ** float(s) and t[s - 1, 1] == (1 - 0.999 ** float(s)) ** 0.5
    assert tuple(t[-1]) == (1.0, 1.0)
