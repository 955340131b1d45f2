"""Parity of the BASELINE configurations beyond C2 against the CPU oracle.

C4 (bf16 mixed precision: bf16 MFMA operands, fp32 accumulate / master weights / activations / norms):
  the reduced operand precision (8-bit mantissa, relative rounding 2^-9) is the only difference from
  fp32, so the bar is the bf16 one:
    forward eps         max|d| vs the fp32 oracle within 1.5x that of the oracle under bf16 operand rounding
    parameter grads     vs an fp64 oracle, relative L2 per tensor: max and median over tensors within
                        1.5x of those of the oracle run with the same bf16 operand rounding (every
                        3x3 conv's input and weights rounded to bf16, fp32 accumulate).  The network is
                        ill-conditioned by construction (ReLU / MaxPool kinks flip under operand
                        rounding, see test_gpu_model.py), so bf16 operand noise alone gives the
                        reference itself relative-L2 gradient errors of ~0.45 (max) / ~0.27 (median)
                        on this input: the bar is "no worse than bf16 autocast of the reference".
    CFG sampler, T=10   max|d| <= 5e-2 * max|ref| on the reference's golden trajectories (w in {0,1,3})
C5 (256x256 maps: up0 = ConvTranspose2d(k=64) on the 1x1 map, AvgPool2d(64)): the fp32 / x6 bar of
  test_gpu_model.py — forward max|d| <= 2e-4 * max|ref| (train and eval BN), grads relative L2 <= 1e-2
  vs fp64 (same rationale as test_train_grads_random_weights_nf64), at n_feat=16, B=1; and at the config's
  own n_feat=256 (B=1, h3 — the shipped arithmetic: 128/256-channel convs on the LDS-halo kernel at
  W = 256 / 128 / 64, BN backward fused at 128^2 and 64^2): forward train / eval vs the fp32 oracle, grads vs
  an fp64 oracle (~1.2 TFLOP per forward on the host: tens of seconds).
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import ref_cpu as R
import _parity

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _model(nf, H=64, seed=0, math="fp32"):
    from cdm_amd import ContextUnet
    torch.manual_seed(seed)
    return ContextUnet(1, nf, 6, H, conv_math=math).cuda()


def _rel(got, ref):
    got = got.detach().double().cpu(); ref = ref.detach().double().cpu()
    return (got - ref).abs().max().item() / max(ref.abs().max().item(), 1e-30)


def _forward_pair(nf, H, B, math, seed=3):
    m = _model(nf, H, seed=seed, math=math)
    g = torch.Generator().manual_seed(9)
    x = torch.rand(B, 1, H, H, generator=g); t = torch.rand(B, generator=g); c = torch.rand(B, 6, generator=g)
    sd = R.clone_sd(m.state_dict())
    out = []
    for train in (False, True):
        m.train(train)
        with torch.no_grad():
            torch.manual_seed(21)
            eps = m(x.cuda(), t.cuda(), c.cuda())
        torch.manual_seed(21)
        ref = R.unet_forward(R.clone_sd(sd), x, t, c, n_feat=nf, n_cfeat=6, height=H, train=train,
                             shortcut=lambda: R.draw_shortcut(1, nf))
        out.append((train, eps, ref))
    return out


from _bf16emu import _RoundBF16, _bf16_operands  # noqa: E402,F401  (shared with tests/golden/make_golden_r5_c4.py)


def _grad_errors(nf, H, B, math, seed=4, emulate_bf16=False):
    T = 1500
    m = _model(nf, H, seed=seed, math=math).train()
    sd = R.clone_sd(m.state_dict())
    g = torch.Generator().manual_seed(10)
    x = torch.rand(B, 1, H, H, generator=g); noise = torch.randn(B, 1, H, H, generator=g)
    c = torch.rand(B, 6, generator=g); tt = torch.randint(1, T + 1, (B,), generator=g)
    _, _, ab = R.make_schedule(T)
    xp = R.perturb_input(x, tt, noise, ab)
    torch.manual_seed(33)
    pred = m(xp.cuda(), (tt / T).cuda(), c.cuda())
    F.mse_loss(pred, noise.cuda()).backward()

    def oracle(dtype):
        s = {k: (v.to(dtype) if v.is_floating_point() else v.clone()) for k, v in sd.items()}
        tr = R.OracleTrainer(s, n_feat=nf, n_cfeat=6, height=H)
        torch.manual_seed(33)
        w, b = R.draw_shortcut(1, nf)
        _, p, gr = tr.step(x.to(dtype), c.to(dtype), noise.to(dtype), tt, T, ab.to(dtype), (w.to(dtype), b.to(dtype)))
        return p, gr

    p64, g64 = oracle(torch.float64)
    gmax = max(v.abs().max().item() for v in g64.values())
    got = {k: p.grad.cpu().double() for k, p in m.named_parameters()}
    emu = None
    if emulate_bf16:
        with _bf16_operands(outputs=True):
            _, emu = oracle(torch.float32)
    errs, errs_emu, zero_ok = {}, {}, True
    for k, v in got.items():
        if ".conv1.0.bias" in k or ".conv2.0.bias" in k:      # analytic gradient 0 (BatchNorm follows)
            zero_ok &= v.abs().max().item() <= 1e-3 * gmax
        else:
            errs[k] = ((v - g64[k]).norm() / g64[k].norm()).item()
            if emu is not None:
                errs_emu[k] = ((emu[k].double() - g64[k]).norm() / g64[k].norm()).item()
    return _rel(pred, p64), errs, zero_ok, errs_emu


# ------------------------------------------------------------------------------------------ C4 (bf16)
def test_c4_bf16_forward_vs_oracle():
    """bf16 forward vs the fp32 oracle: within 1.5x the error of the oracle itself under bf16 operand rounding
    (train-mode BatchNorm amplifies operand noise: ~2 % of max|eps| for both on this input)."""
    got = _forward_pair(64, 64, 3, "bf16")
    with _bf16_operands():                   # eval: operands rounded (the eval forward keeps fp32 activations)
        emu = _forward_pair(64, 64, 3, "fp32")
    with _bf16_operands(outputs=True):       # train: the fused chain's y also stored in bf16, as autocast does
        emu_t = _forward_pair(64, 64, 3, "fp32")
    emu = [emu[0], emu_t[1]]
    for (train, eps, ref), (_, _, ref_bf) in zip(got, emu):
        e_hip, e_emu = _rel(eps, ref), _rel(ref_bf, ref)
        print("train" if train else "eval", "hip", e_hip, "oracle-bf16", e_emu)
        assert e_hip <= max(1.5 * e_emu, 1e-3), (train, e_hip, e_emu)


def test_c4_bf16_train_grads_vs_fp64():
    perr, errs, zero_ok, emu = _grad_errors(64, 64, 2, "bf16", emulate_bf16=True)
    worst = sorted(errs.items(), key=lambda kv: kv[1])[-5:]
    print("pred rel", perr, "worst grads", worst, "oracle-bf16 max", max(emu.values()),
          "median", float(np.median(list(emu.values()))))
    assert perr < 2e-2
    assert zero_ok
    assert max(errs.values()) <= 1.5 * max(emu.values()), worst
    assert float(np.median(list(errs.values()))) <= 1.5 * float(np.median(list(emu.values())))


@pytest.mark.parametrize("w", [0.0, 1.0, 3.0])
def test_c4_bf16_cfg_sampler_vs_reference_golden(w):
    import cdm_amd
    fx = np.load(os.path.join(GOLD, "model_nf8.npz"))
    sd = {k[3:]: torch.from_numpy(fx[k].copy()) for k in fx.files if k.startswith("sd.")}
    m = cdm_amd.ContextUnet(1, 8, 6, 64, conv_math="bf16")
    m.load_state_dict(sd)
    m = m.cuda().eval()
    sfx = np.load(os.path.join(GOLD, "sampler_nf8.npz"))
    d = cdm_amd.DDPM(m, int(sfx["T"]), "cuda", z_source="host", sched_tensors=_parity.golden_schedule(int(sfx["T"])))
    torch.manual_seed(500)                       # the reference's RNG state for this trajectory
    x, inter = d.sample_ddpm(2, 64, None, torch.from_numpy(sfx["params"]), w)
    # bar: 1.5x the error of the reference's own sampler under the same bf16 operand rounding (the CPU oracle, which
    # replays the reference's RNG order bit-exactly, with every 3x3 conv's operands rounded to bf16), at least 1e-3
    T = int(sfx["T"])
    with _bf16_operands():
        torch.manual_seed(500)
        xe, inte = R.sample_ddpm(R.make_model_fn(R.clone_sd(sd), n_feat=8, n_cfeat=6, height=64), 2, 64,
                                 torch.from_numpy(sfx["params"]), w, T, _parity.golden_schedule(T), 6)
    gx, gi = torch.from_numpy(sfx[f"sample_w{w:g}"]), torch.from_numpy(sfx[f"sample_w{w:g}_inter"])
    e_hip, e_emu = _rel(x, gx), _rel(xe, gx)
    ei_hip, ei_emu = _rel(torch.from_numpy(inter), gi), _rel(inte, gi)
    print(f"w={w:g}: final hip {e_hip:.2e} oracle-bf16 {e_emu:.2e}; snapshots hip {ei_hip:.2e} oracle-bf16 {ei_emu:.2e}")
    assert e_hip <= max(1.5 * e_emu, 1e-3), (e_hip, e_emu)
    assert ei_hip <= max(1.5 * ei_emu, 1e-3), (ei_hip, ei_emu)


def test_c4_bf16_trainer_step_vs_emulated_oracle():
    """The C4 Trainer step bench.py times (bf16 arithmetic, fused BN / ConvT paths, Adam), one injected step at nf=64,
    B=4: gradients and post-Adam parameters vs the fp64 oracle within 1.5x the error of the reference run under the
    same bf16 operand rounding (_bf16_operands), the bar of test_c4_bf16_train_grads_vs_fp64 (statistics over every
    parameter); the loss, one scalar whose bf16 error is a random-sign sum over the batch, within 3x the emulated
    reference's (measured 2.2x)."""
    from cdm_amd import Trainer
    nf, B, T, lr = 64, 4, 1500, 1e-4
    m = _model(nf, seed=7, math="bf16").train()
    sd = R.clone_sd(m.state_dict())
    g = torch.Generator().manual_seed(31)
    x = torch.rand(B, 1, 64, 64, generator=g); c = torch.rand(B, 6, generator=g)
    noise = torch.randn(B, 1, 64, 64, generator=g); tt = torch.randint(1, T + 1, (B,), generator=g)
    sc = torch.rand(2 * nf, generator=g) * 2 - 1
    tr = Trainer(m, lr, T, B, use_graph=False)
    loss = float(tr.step(x.cuda(), c.cuda(), inject=(noise.cuda(), tt.cuda().int(), sc.cuda())).item())
    torch.cuda.synchronize()
    grads = {n: v.detach().cpu().double() for n, v in tr.grads.items()}
    post = {n: v.detach().cpu().double() for n, v in tr.views.items()}
    _, _, ab = R.make_schedule(T)

    def oracle(dtype, emulate):
        s = {k: (v.to(dtype) if v.is_floating_point() else v.clone()) for k, v in sd.items()}
        otr = R.OracleTrainer(s, n_feat=nf, n_cfeat=6, height=64, lr=lr)
        w, b = sc[:nf].reshape(nf, 1, 1, 1).to(dtype), sc[nf:].to(dtype)
        args = (x.to(dtype), c.to(dtype), noise.to(dtype), tt, T, ab.to(dtype), (w, b))
        if emulate:
            with _bf16_operands(outputs=True):
                l, _, gr = otr.step(*args)
        else:
            l, _, gr = otr.step(*args)
        return float(l), gr, {k: v.detach().clone() for k, v in otr.sd.items()}
    l64, g64, sd64 = oracle(torch.float64, False)
    le, ge, sde = oracle(torch.float32, True)
    keep = [n for n in grads if not (".conv1.0.bias" in n or ".conv2.0.bias" in n)]
    eh = {n: ((grads[n] - g64[n]).norm() / g64[n].norm()).item() for n in keep}
    ee = {n: ((ge[n].double() - g64[n]).norm() / g64[n].norm()).item() for n in keep}
    dh = np.concatenate([((post[n] - sd64[n]) / lr).abs().numpy().ravel() for n in keep])
    de = np.concatenate([((sde[n].double() - sd64[n]) / lr).abs().numpy().ravel() for n in keep])
    rh, re_ = float(np.sqrt((dh ** 2).mean())), float(np.sqrt((de ** 2).mean()))
    res = dict(loss_err=abs(loss - l64), loss_err_emulated=abs(le - l64), grad_max=max(eh.values()),
               grad_max_emulated=max(ee.values()), grad_median=float(np.median(list(eh.values()))),
               grad_median_emulated=float(np.median(list(ee.values()))), param_dev_lr_rms=rh,
               param_dev_lr_rms_emulated=re_)
    _parity.record("c4_bf16_trainer_step", n_feat=nf, B=B, **res)
    print(res)
    assert res["loss_err"] <= 3 * res["loss_err_emulated"] + 1e-6
    assert res["grad_max"] <= 1.5 * res["grad_max_emulated"]
    assert res["grad_median"] <= 1.5 * res["grad_median_emulated"]
    assert rh <= 1.5 * re_ + 1e-3


@pytest.mark.parametrize("w", [0.0, 3.0])
def test_c4_bf16_cfg_T1500_vs_emulated_oracle(w):
    """bf16 sampling at the benchmarked T=1500 (w=0 and the CFG w=3), CPU-RNG replay of the reference's run
    (tests/golden/sampler_T1500_nf8.npz): the deviation from the reference's fp64 trajectory, RMS over the final x and
    the 13 stored snapshots (each relative to its max|x|), within 1.5x that of the reference's own sampler run under
    the same bf16 operand rounding (the CPU oracle with _bf16_operands, same RNG replay), at least 1e-3."""
    import cdm_amd
    sfx = np.load(os.path.join(GOLD, "sampler_T1500_nf8.npz"))
    T = int(sfx["T"])
    fx = np.load(os.path.join(GOLD, "model_nf8.npz"))
    sd = {k[3:]: torch.from_numpy(fx[k].copy()) for k in fx.files if k.startswith("sd.")}
    m = cdm_amd.ContextUnet(1, 8, 6, 64, conv_math="bf16")
    m.load_state_dict(sd)
    m = m.cuda().eval()
    d = cdm_amd.DDPM(m, T, "cuda", z_source="host", sched_tensors=_parity.golden_schedule(T))
    seed = int(sfx[f"w{w:g}_seed"])
    torch.manual_seed(seed)
    x, inter = d.sample_ddpm(2, 64, None, torch.from_numpy(sfx["params"]), w)
    with _bf16_operands():
        torch.manual_seed(seed)
        xe, inte = R.sample_ddpm(R.make_model_fn(R.clone_sd(sd), n_feat=8, n_cfeat=6, height=64), 2, 64,
                                 torch.from_numpy(sfx["params"]), w, T, _parity.golden_schedule(T), 6)
    keep = sfx["snap_keep"]

    def errs(final, snaps):
        out = [float(np.abs(np.asarray(final) - sfx[f"w{w:g}_x_fp64"]).max() / np.abs(sfx[f"w{w:g}_x_fp64"]).max())]
        for j, s in enumerate(keep):
            r = sfx[f"w{w:g}_inter_fp64"][j]
            out.append(float(np.abs(np.asarray(snaps[s]) - r).max() / np.abs(r).max()))
        return np.array(out)
    eh = errs(x.cpu().numpy(), inter)
    ee = errs(xe.numpy(), inte.numpy())
    rh, re_ = float(np.sqrt((eh ** 2).mean())), float(np.sqrt((ee ** 2).mean()))
    _parity.record("c4_bf16_sample_T1500", w=w, rms_err=rh, rms_err_emulated=re_, final_err=float(eh[0]),
                   final_err_emulated=float(ee[0]))
    print(f"T=1500 bf16 w={w:g}: RMS deviation from fp64 HIP {rh:.3e}, emulated reference {re_:.3e}; final "
          f"{eh[0]:.3e} / {ee[0]:.3e}")
    assert rh <= max(1.5 * re_, 1e-3)


@pytest.mark.parametrize("w", [0.0, 3.0])
def test_c4_bf16_nf128_T1500_vs_emulated_reference(w):
    """C4's benchmarked trajectories: bf16 sampling at n_feat = 128, T = 1500, w = 0 and the CFG w = 3 (the goldens of
    test_sample_nf128_T1500_matches_reference: seeded init, n = 2, the golden's schedule, b_t.sqrt() table and CPU-RNG
    draws).  Bar: the deviation from the golden's fp64 re-run, RMS over the final x and the 13 stored snapshots (each
    relative to its max|x|), within 1.5x that of the reference's own sampler under C4's bf16 operand rounding (the CPU
    oracle under _bf16_operands, same draws, precomputed by tests/golden/make_golden_r5_c4.py), at least 1e-3."""
    import cdm_amd
    k = f"w{w:g}"
    g = np.load(os.path.join(GOLD, "sampler_T1500_nf128.npz" if w == 0 else f"sampler_T1500_nf128_{k}.npz"))
    e = np.load(os.path.join(GOLD, "sampler_T1500_nf128_bf16emu.npz" if w == 0 else f"sampler_T1500_nf128_{k}_bf16emu.npz"))
    T, nf = int(g["T"]), int(g["n_feat"])
    torch.manual_seed(int(g["init_seed"]))
    m = cdm_amd.ContextUnet(1, nf, 6, 64, conv_math="bf16").cuda().eval()
    d = cdm_amd.DDPM(m, T, "cuda", z_source="host", sched_tensors=_parity.golden_schedule(T),
                     sched_sb=_parity.golden_sqrt_b(T))
    torch.manual_seed(int(g[f"{k}_seed"]))
    x, inter = d.sample_ddpm(2, 64, None, torch.from_numpy(g["params"]), w)
    keep = [int(s) for s in g["snap_keep"]]

    def errs(final, snaps):
        out = [float(np.abs(np.asarray(final, np.float64) - g[f"{k}_x_fp64"]).max() / np.abs(g[f"{k}_x_fp64"]).max())]
        for j in range(len(keep)):
            r = g[f"{k}_inter_fp64"][j]
            out.append(float(np.abs(np.asarray(snaps[j], np.float64) - r).max() / np.abs(r).max()))
        return np.array(out)
    eh = errs(x.cpu().numpy(), [inter[s] for s in keep])
    ee = errs(e[f"{k}_x_bf16emu"], e[f"{k}_inter_bf16emu"])
    rh, re_ = float(np.sqrt((eh ** 2).mean())), float(np.sqrt((ee ** 2).mean()))
    _parity.record("c4_bf16_sample_nf128_T1500", w=w, rms_err=rh, rms_err_emulated=re_, final_err=float(eh[0]),
                   final_err_emulated=float(ee[0]))
    print(f"C4 nf128 T=1500 w={w:g}: RMS deviation from fp64 HIP {rh:.3e}, emulated reference {re_:.3e}; final "
          f"{eh[0]:.3e} / {ee[0]:.3e}")
    assert rh <= max(1.5 * re_, 1e-3)


# ------------------------------------------------------------------------------------------ C5 (256x256)
@pytest.mark.parametrize("math", ["fp32", "x6", "h3"])
def test_c5_256_forward_vs_oracle(math):
    for train, eps, ref in _forward_pair(16, 256, 1, math):
        assert _rel(eps, ref) < 2e-4, (train, _rel(eps, ref))


@pytest.mark.parametrize("math", ["x6", "h3"])
def test_c5_256_train_grads_vs_fp64(math):
    """h3 at 256x256 runs the wide-row LDS-halo kernel (W 256 / 128) and, at 128x128, the fused BN backward."""
    perr, errs, zero_ok, _ = _grad_errors(16, 256, 1, math)
    worst = sorted(errs.items(), key=lambda kv: kv[1])[-5:]
    print("pred rel", perr, "worst grads", worst)
    assert perr < 2e-4
    assert zero_ok
    assert max(errs.values()) <= 1e-2, worst
    assert float(np.median(list(errs.values()))) <= 5e-3


def test_c5_nf256_forward_vs_oracle():
    """C5's own width: n_feat=256 at 256x256 (h3), forward in train and eval BatchNorm vs the fp32 oracle."""
    for train, eps, ref in _forward_pair(256, 256, 1, "h3"):
        print("train" if train else "eval", _rel(eps, ref))
        assert _rel(eps, ref) < 2e-4, (train, _rel(eps, ref))


def _grad_errors_fp64_light(nf, H, B, math, seed=4):
    """_grad_errors without the oracle's Adam state and gradient copies (C5 at n_feat=256 has 1.09 G parameters:
    up0's ConvTranspose2d(512, 512, 64) alone is 1.07 G): fp64 forward + backward on leaf tensors, compared
    tensor by tensor."""
    T = 1500
    m = _model(nf, H, seed=seed, math=math).train()
    g = torch.Generator().manual_seed(10)
    x = torch.rand(B, 1, H, H, generator=g); noise = torch.randn(B, 1, H, H, generator=g)
    c = torch.rand(B, 6, generator=g); tt = torch.randint(1, T + 1, (B,), generator=g)
    _, _, ab = R.make_schedule(T)
    xp = R.perturb_input(x, tt, noise, ab)
    torch.manual_seed(33)
    pred = m(xp.cuda(), (tt / T).cuda(), c.cuda())
    F.mse_loss(pred, noise.cuda()).backward()
    keys = [k for k, _, kind in R.state_dict_layout(1, nf, 6, H) if kind == "param"]
    s = {k: (v.detach().cpu().double() if v.is_floating_point() else v.detach().cpu().clone())
         for k, v in m.state_dict().items()}
    for k in keys:
        s[k].requires_grad_(True)
    torch.manual_seed(33)
    w, b = R.draw_shortcut(1, nf)
    p64 = R.unet_forward(s, R.perturb_input(x.double(), tt, noise.double(), ab.double()), (tt / T).double(), c.double(),
                         train=True, shortcut=(w.double(), b.double()), n_feat=nf, n_cfeat=6, height=H)
    F.mse_loss(p64, noise.double()).backward()
    gmax = max(s[k].grad.abs().max().item() for k in keys)
    params = dict(m.named_parameters())
    errs, zero_ok = {}, True
    for k in keys:
        v, ref = params[k].grad.detach().cpu().double(), s[k].grad
        if ".conv1.0.bias" in k or ".conv2.0.bias" in k:      # analytic gradient 0 (BatchNorm follows)
            zero_ok &= v.abs().max().item() <= 1e-3 * gmax
        else:
            errs[k] = ((v - ref).norm() / ref.norm()).item()
        s[k].grad = None
    return _rel(pred, p64), errs, zero_ok


def test_c5_nf256_train_grads_vs_fp64():
    """C5's own width: every parameter gradient of one train step (n_feat=256, 256x256, B=1, h3) vs fp64."""
    perr, errs, zero_ok = _grad_errors_fp64_light(256, 256, 1, "h3")
    worst = sorted(errs.items(), key=lambda kv: kv[1])[-5:]
    print("pred rel", perr, "worst grads", worst, "median", float(np.median(list(errs.values()))))
    assert perr < 2e-4
    assert zero_ok
    assert max(errs.values()) <= 1e-2, worst
    assert float(np.median(list(errs.values()))) <= 5e-3


def test_c4_bf16_eval_under_autograd_matches_no_grad_eval():
    """model.eval() under autograd (the train-structured forward with BatchNorm frozen on the running
    statistics) keeps fp32 activations under C4's bf16 arithmetic, like the no-grad eval path, so the same eval model
    returns eps of the same accuracy whether or not autograd records it.  n_feat = 128 (the width whose fused chain
    stores bf16 activations in train mode), B = 2: eps with and without grad, and the input / parameter gradients, vs
    fp64 autograd of the oracle in eval mode, within 1.5x the oracle run under the same bf16 operand rounding."""
    nf, B, H = 128, 2, 64
    m = _model(nf, H, seed=5, math="bf16").eval()
    sd = R.clone_sd(m.state_dict())
    g = torch.Generator().manual_seed(19)
    x = torch.randn(B, 1, H, H, generator=g); t = torch.rand(B, generator=g); c = torch.rand(B, 6, generator=g)
    wgt = torch.randn(B, 1, H, H, generator=g)
    with torch.no_grad():
        torch.manual_seed(21)
        eps_ng = m(x.cuda(), t.cuda(), c.cuda()).cpu()
    xg = x.cuda().requires_grad_(True)
    torch.manual_seed(21)
    eps_g = m(xg, t.cuda(), c.cuda())
    (eps_g * wgt.cuda()).sum().backward()
    keys = [k for k, _, kind in R.state_dict_layout(1, nf, 6, H) if kind == "param"]

    def oracle(dtype):
        s = {k: (v.to(dtype) if v.is_floating_point() else v.clone()).clone() for k, v in sd.items()}
        for k in keys:
            s[k].requires_grad_(True)
        xx = x.to(dtype).clone().requires_grad_(True)
        torch.manual_seed(21)
        w_, b_ = R.draw_shortcut(1, nf)
        e = R.unet_forward(s, xx, t.to(dtype), c.to(dtype), n_feat=nf, n_cfeat=6, height=H, train=False,
                           shortcut=(w_.to(dtype), b_.to(dtype)))
        (e * wgt.to(dtype)).sum().backward()
        return e.detach(), xx.grad, {k: s[k].grad for k in keys}
    e64, dx64, g64 = oracle(torch.float64)
    with _bf16_operands():
        eem, dxem, gem = oracle(torch.float32)
    e_ng, e_g, e_em = _rel(eps_ng, e64), _rel(eps_g, e64), _rel(eem, e64)
    rl2 = lambda a, b: ((a.detach().double().cpu() - b.double()).norm() / b.double().norm()).item()   # noqa: E731
    errs = {k: rl2(p.grad, g64[k]) for k, p in m.named_parameters() if g64[k].norm() > 0}
    errs_em = {k: rl2(gem[k], g64[k]) for k in errs}
    dx_err, dx_em = rl2(xg.grad.view(B, 1, H, H), dx64), rl2(dxem, dx64)
    print(f"eval bf16 eps no-grad {e_ng:.2e} / grad {e_g:.2e} / emulated {e_em:.2e}; dx {dx_err:.2e} / {dx_em:.2e}; "
          f"grads max {max(errs.values()):.2e} / {max(errs_em.values()):.2e}")
    _parity.record("c4_eval_under_autograd", eps_no_grad=e_ng, eps_grad=e_g, eps_emulated=e_em, dx=dx_err,
                   dx_emulated=dx_em, grad_max=max(errs.values()), grad_max_emulated=max(errs_em.values()))
    assert e_ng <= 1.5 * e_em and e_g <= 1.5 * e_em
    assert dx_err <= 1.5 * dx_em
    assert max(errs.values()) <= 1.5 * max(errs_em.values())
    assert float(np.median(list(errs.values()))) <= 1.5 * float(np.median(list(errs_em.values())))
