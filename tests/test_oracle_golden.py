"""Pin the CPU oracle to golden vectors produced by the reference itself (tests/golden/make_golden.py).

All comparisons are bit-exact: the oracle runs the same fp32 CPU operators in the same order and
replays the reference's CPU RNG consumption (x_T, per-step z, per-forward random shortcut)."""
import os

import numpy as np
import pytest
import torch

from oracle import ref_cpu as R



@pytest.fixture(autouse=True)
def _eight_threads():
    """The golden vectors were produced with 8 intra-op threads; CPU conv reductions are split per
    thread, so bit-exactness holds at exactly that partitioning."""
    old = torch.get_num_threads()
    torch.set_num_threads(8)
    yield
    torch.set_num_threads(old)


def _load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name))


def _sd(fx, prefix="sd."):
    return {k[len(prefix):]: torch.from_numpy(fx[k].copy()) for k in fx.files if k.startswith(prefix)}


def test_schedule_bit_exact(golden_dir):
    fx = _load(golden_dir, "schedule.npz")
    for T in (1000, 1500, 2000):
        b, a, ab = R.make_schedule(T)
        assert np.array_equal(b.numpy(), fx[f"b_t_{T}"])
        assert np.array_equal(a.numpy(), fx[f"a_t_{T}"])
        assert np.array_equal(ab.numpy(), fx[f"ab_t_{T}"])


@pytest.mark.parametrize("nf", [8, 16])
def test_layout_matches_reference(golden_dir, nf):
    fx = _load(golden_dir, f"model_nf{nf}.npz")
    sd = _sd(fx)
    layout = R.state_dict_layout(1, nf, 6, 64)
    assert [k for k, _, _ in layout] == list(sd.keys())
    for k, shape, _ in layout:
        assert tuple(sd[k].shape) == shape, k


def test_layout_nf128_metadata(golden_dir):
    import json
    meta = json.load(open(os.path.join(golden_dir, "layout_nf128.json")))
    layout = R.state_dict_layout(1, 128, 6, 64)
    assert [k for k, _, _ in layout] == [k for k, _, _ in meta["keys"]]
    assert [list(s) for _, s, _ in layout] == [s for _, s, _ in meta["keys"]]
    n = sum(int(np.prod(s)) for _, s, kind in layout if kind == "param")
    assert n == meta["n_params"] == 21626881


@pytest.mark.parametrize("nf", [8, 16])
def test_eval_forward_bit_exact(golden_dir, nf):
    fx = _load(golden_dir, f"model_nf{nf}.npz")
    sd = _sd(fx)
    x, t, c = (torch.from_numpy(fx[k]) for k in ("x", "t", "c"))
    sc = (torch.from_numpy(fx["eval_sc_w"]), torch.from_numpy(fx["eval_sc_b"]))
    eps = R.unet_forward(sd, x, t, c, n_feat=nf, n_cfeat=6, height=64, train=False, shortcut=sc)
    assert np.array_equal(eps.numpy(), fx["eval_eps"])
    # unconditional, scalar t broadcast (train_diffusion.py:186)
    sc = (torch.from_numpy(fx["eval_uncond_sc_w"]), torch.from_numpy(fx["eval_uncond_sc_b"]))
    t1 = torch.from_numpy(fx["t1"])[:, None, None, None]
    eps = R.unet_forward(sd, x, t1, None, n_feat=nf, n_cfeat=6, height=64, train=False, shortcut=sc)
    assert np.array_equal(eps.numpy(), fx["eval_uncond_eps"])


def test_shortcut_draw_replays_cpu_rng(golden_dir):
    fx = _load(golden_dir, "model_nf8.npz")
    torch.manual_seed(11)
    w, b = R.draw_shortcut(1, 8)
    assert np.array_equal(w.numpy(), fx["eval_sc_w"]) and np.array_equal(b.numpy(), fx["eval_sc_b"])


def test_train_steps_bit_exact(golden_dir):
    fx = _load(golden_dir, "model_nf8.npz")
    nf, T = 8, int(fx["train_T"])
    sd = _sd(fx)
    x, c = torch.from_numpy(fx["x"]), torch.from_numpy(fx["c"])
    _, _, ab_t = R.make_schedule(T)
    tr = R.OracleTrainer(sd, n_feat=nf, n_cfeat=6, height=64, lr=1e-3)
    for step in range(2):
        torch.manual_seed(100 + step)          # same RNG order as the reference loop body
        noise = torch.randn_like(x)
        tt = torch.randint(1, T + 1, (x.shape[0],))
        draw = lambda: R.draw_shortcut(1, nf)
        loss, pred, grads = tr.step(x, c, noise, tt, T, ab_t, draw)
        if step == 0:
            assert np.array_equal(noise.numpy(), fx["train0_noise"])
            assert np.array_equal(tt.numpy(), fx["train0_t"])
            assert np.array_equal(pred.numpy(), fx["train0_eps"])
            assert loss.item() == float(fx["train0_loss"])
            for k, g in grads.items():
                assert np.array_equal(g.numpy(), fx["train0_grad." + k]), k
    for k in tr.sd:
        assert np.array_equal(tr.sd[k].detach().numpy(), fx["after2." + k]), k


@pytest.mark.parametrize("w", [0.0, 1.0, 3.0])
def test_sampler_cfg_bit_exact(golden_dir, w):
    sfx = _load(golden_dir, "sampler_nf8.npz")
    sd = _sd(_load(golden_dir, "model_nf8.npz"))
    T = int(sfx["T"])
    sched = R.make_schedule(T)
    fn = R.make_model_fn(sd, n_feat=8, n_cfeat=6, height=64)
    torch.manual_seed(500)
    xs, inter = R.sample_ddpm(fn, 2, 64, torch.from_numpy(sfx["params"]), w, T, sched, n_cfeat=6)
    assert np.array_equal(xs.numpy(), sfx[f"sample_w{w:g}"])
    assert np.array_equal(inter.numpy(), sfx[f"sample_w{w:g}_inter"])


def test_sampler_random_params_and_from_noise(golden_dir):
    sfx = _load(golden_dir, "sampler_nf8.npz")
    sd = _sd(_load(golden_dir, "model_nf8.npz"))
    T = int(sfx["T"])
    sched = R.make_schedule(T)
    fn = R.make_model_fn(sd, n_feat=8, n_cfeat=6, height=64)
    torch.manual_seed(501)
    xs, _ = R.sample_ddpm(fn, 2, 64, None, 0.0, T, sched, n_cfeat=6)
    assert np.array_equal(xs.numpy(), sfx["sample_noparams"])
    x0 = torch.from_numpy(sfx["fromnoise_x0"])
    noise = torch.from_numpy(sfx["fromnoise_noise"])
    xT = R.perturb_input(x0, T, noise, sched[2])
    assert np.array_equal(xT.numpy(), sfx["fromnoise_xT"])
    torch.manual_seed(502)
    torch.randn_like(x0)  # the reference drew `noise` from this seed first
    xs, inter = R.sample_ddpm_from_noise(fn, xT, torch.from_numpy(sfx["params"]), 1.0, T, sched)
    assert np.array_equal(xs.numpy(), sfx["fromnoise_out"])
    assert np.array_equal(inter.numpy(), sfx["fromnoise_inter"])


def test_forward_flops_matches_survey():
    assert abs(R.forward_flops(128, 64) / 1e9 - 19.178788) < 2e-3


def _lik_batches(lfx):
    return [(torch.from_numpy(lfx[f"lik_x{j}"]), torch.from_numpy(lfx[f"lik_c{j}"])) for j in range(2)]


def test_likelihood_and_elbo_bit_exact(golden_dir):
    """next-1: the NLL estimator (both scripts) and the dataset ELBO/BPD, CPU RNG order."""
    lfx = _load(golden_dir, "likelihood_nf8.npz")
    sd = _sd(_load(golden_dir, "model_nf8.npz"))
    fn = R.make_model_fn(sd, n_feat=8, n_cfeat=6, height=64)
    T = int(lfx["T_lik"])
    torch.manual_seed(600)
    nll = R.calculate_likelihood(fn, _lik_batches(lfx), T, R.make_schedule(T))
    assert nll == float(lfx["nll_elbo_script"]) == float(lfx["nll_paper_script"])
    T = int(lfx["T_elbo"])
    torch.manual_seed(601)
    elbo, bpd = R.calculate_elbo_and_bpd_dataset(fn, _lik_batches(lfx), T, R.make_schedule(T))
    assert elbo == float(lfx["paper_elbo"]) and bpd == float(lfx["paper_bpd"])


def test_batch_elbo_bit_exact(golden_dir):
    lfx = _load(golden_dir, "likelihood_nf8.npz")
    b, a, ab = R.make_schedule(int(lfx["T_elbo"]))
    g = lambda k: torch.from_numpy(lfx[k])
    e, bp = R.calculate_elbo_and_bpd_batch(g("batch_x"), g("batch_pred"), g("batch_noise"), g("batch_t"), b, a, ab,
                                           64 * 64)
    assert e.item() == float(lfx["batch_elbo"]) and bp.item() == float(lfx["batch_bpd"])


def test_train_loop_with_lr_decay_bit_exact(golden_dir):
    """train_nf8.npz (make_golden_r2.py): three reference loop iterations incl. the per-epoch LR change — the
    oracle's OracleTrainer reproduces every post-step state_dict (parameters, BN buffers) bit for bit."""
    fx = np.load(os.path.join(golden_dir, "train_nf8.npz"))
    base = np.load(os.path.join(golden_dir, "model_nf8.npz"))
    sd = {k[3:]: torch.from_numpy(base[k].copy()) for k in base.files if k.startswith("sd.")}
    T = int(fx["T"])
    _, _, ab = R.make_schedule(T)
    tr = R.OracleTrainer(sd, n_feat=8, n_cfeat=6, height=64, lr=float(fx["lrate"]))
    x, c = torch.from_numpy(fx["x"]), torch.from_numpy(fx["c"])
    for k in range(3):
        w = torch.from_numpy(fx[f"s{k}_sc_w"]).reshape(8, 1, 1, 1)
        b = torch.from_numpy(fx[f"s{k}_sc_b"])
        loss, _, g = tr.step(x, c, torch.from_numpy(fx[f"s{k}_noise"]), torch.from_numpy(fx[f"s{k}_t"]), T, ab, (w, b),
                             lr=float(fx[f"s{k}_lr"]))
        assert float(loss) == float(fx[f"s{k}_loss"])
        if k == 0:
            for n, v in g.items():
                assert np.array_equal(v.numpy(), fx["s0_grad." + n]), n
        for n, v in tr.sd.items():
            assert np.array_equal(v.detach().numpy(), fx[f"s{k}_after.{n}"]), (k, n)
    assert [float(fx[f"s{k}_lr"]) for k in range(3)] == [1e-3, 1e-3, 7.5e-4]


def test_sampler_T1500_bit_exact(golden_dir):
    """sampler_T1500_nf8.npz, w=0: the oracle's sample_loop replays the reference's 1500-step CPU run bit for bit
    (x_T, 1499 z and 1500 shortcut draws from the CPU RNG)."""
    fx = np.load(os.path.join(golden_dir, "sampler_T1500_nf8.npz"))
    base = np.load(os.path.join(golden_dir, "model_nf8.npz"))
    sd = {k[3:]: torch.from_numpy(base[k].copy()) for k in base.files if k.startswith("sd.")}
    T = int(fx["T"])
    torch.manual_seed(int(fx["w0_seed"]))
    fn = R.make_model_fn(sd, n_feat=8, n_cfeat=6, height=64)
    x, inter = R.sample_ddpm(fn, 2, 64, torch.from_numpy(fx["params"]), 0.0, T, R.make_schedule(T), 6)
    assert np.array_equal(x.numpy(), fx["w0_x"])
    assert np.array_equal(inter.numpy()[list(fx["snap_keep"])], fx["w0_inter"])
