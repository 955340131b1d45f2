"""Sampler parity (a9-a12) on the GPU against the reference's golden trajectories.

z_source="host" replays the reference CPU-run RNG order (x_T, then per step z and the random
shortcut draw(s)), so the only differences are the network's fp32 summation order.
Tolerance: trajectory max|d| <= 1e-3 * max|ref| at T=10 (error grows ~ 1/sqrt(ab_T) per SURVEY §7).
perturb_input / denoise_add_noise on identical inputs are bit-exact (same fp32 op order, no fma).
"""
import os

import numpy as np
import pytest
import torch

from oracle import ref_cpu as R

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _model():
    import cdm_amd
    fx = np.load(os.path.join(GOLD, "model_nf8.npz"))
    sd = {k[3:]: torch.from_numpy(fx[k].copy()) for k in fx.files if k.startswith("sd.")}
    m = cdm_amd.ContextUnet(1, 8, 6, 64)
    m.load_state_dict(sd)
    return m.cuda().eval()


def _rel(a, b):
    a = torch.as_tensor(a).float().cpu(); b = torch.as_tensor(b).float().cpu()
    return (a - b).abs().max().item() / b.abs().max().item()


@pytest.mark.parametrize("w", [0.0, 1.0, 3.0])
def test_sample_ddpm_cfg_matches_reference(w):
    import cdm_amd
    sfx = np.load(os.path.join(GOLD, "sampler_nf8.npz"))
    T = int(sfx["T"])
    d = cdm_amd.DDPM(_model(), T, "cuda", z_source="host")
    torch.manual_seed(500)
    x, inter = d.sample_ddpm(2, 64, None, torch.from_numpy(sfx["params"]), w)
    assert _rel(x, sfx[f"sample_w{w:g}"]) < 1e-3
    assert inter.shape == sfx[f"sample_w{w:g}_inter"].shape
    assert _rel(inter, sfx[f"sample_w{w:g}_inter"]) < 1e-3


def test_sample_random_params_and_from_noise():
    import cdm_amd
    sfx = np.load(os.path.join(GOLD, "sampler_nf8.npz"))
    T = int(sfx["T"])
    d = cdm_amd.DDPM(_model(), T, "cuda", z_source="host")
    torch.manual_seed(501)
    x, _ = d.sample_ddpm(2, 64, None, None, 0.0)
    assert _rel(x, sfx["sample_noparams"]) < 1e-3
    xT = torch.from_numpy(sfx["fromnoise_xT"]).cuda()
    torch.manual_seed(502)
    torch.randn(2, 1, 64, 64)            # the reference drew its forward-diffusion noise here
    x, inter = d.sample_ddpm_from_noise(xT, torch.from_numpy(sfx["params"]), guide_w=1.0)
    assert _rel(x, sfx["fromnoise_out"]) < 1e-3
    assert _rel(inter, sfx["fromnoise_inter"]) < 1e-3


def test_perturb_and_denoise_bit_exact():
    import cdm_amd
    T = 1500
    sched = cdm_amd.Schedule(T, "cuda")
    b, a, ab = R.make_schedule(T)
    g = torch.Generator().manual_seed(3)
    x = torch.rand(4, 1, 64, 64, generator=g); noise = torch.randn(4, 1, 64, 64, generator=g)
    t = torch.tensor([1, 750, 1500, 3])
    ref = R.perturb_input(x, t, noise, ab)
    got = cdm_amd.perturb_input(x.cuda(), t.cuda(), noise.cuda(), sched).cpu()
    assert torch.equal(got, ref)
    ref = R.perturb_input(x, T, noise, ab)                           # scalar t (forward to x_T)
    assert torch.equal(cdm_amd.perturb_input(x.cuda(), T, noise.cuda(), sched).cpu(), ref)
    eps = torch.randn(4, 1, 64, 64, generator=g); z = torch.randn(4, 1, 64, 64, generator=g)
    for i in (1500, 750, 2):
        ref = R.denoise_add_noise(x, i, eps, z, b, a, ab)
        got = cdm_amd.denoise_add_noise(x.cuda(), i, eps.cuda(), z.cuda(), sched).cpu()
        assert torch.equal(got, ref), i
    ref = R.denoise_add_noise(x, 1, eps, 0, b, a, ab)
    assert torch.equal(cdm_amd.denoise_add_noise(x.cuda(), 1, eps.cuda(), 0, sched).cpu(), ref)


def test_graph_replay_equals_eager():
    import cdm_amd
    m = _model()
    sched = cdm_amd.Schedule(30, "cuda")
    params = torch.rand(3, 6, generator=torch.Generator().manual_seed(1))
    outs = []
    for use_graph in (True, False):
        smp = cdm_amd.GraphSampler(m, sched, 3, 3.0, params, z_source="device", seed=11, use_graph=use_graph,
                                   steps_per_graph=7)
        torch.manual_seed(4)
        smp.prepare_rng(host_z=False)
        xT = torch.randn(3, 1, 64, 64, generator=torch.Generator().manual_seed(2))
        x, inter = smp.run(xT)
        outs.append((x.cpu(), inter))
    assert torch.equal(outs[0][0], outs[1][0])
    assert np.array_equal(outs[0][1], outs[1][1])
