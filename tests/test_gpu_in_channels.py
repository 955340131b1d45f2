"""ContextUnet(in_channels > 1) on the HIP engine (ContextUnet.py:6,14,39: init_conv = ResidualConvBlock(in_channels,
n_feat, is_res=True) with its fresh 1x1 shortcut, out.3 = Conv2d(n_feat, in_channels); every reference call site builds
in_channels = 1, whose dedicated kernels the other tests cover).  More image channels run the general conv kernels on
NHWC images padded to a multiple of 4 channels; in_channels == n_feat takes the reference's identity shortcut
(diffusion_utilities.py:50-52, no draw).

Bar (as tests/test_gpu_input_grads.py): HIP vs fp64 autograd of the oracle on HIP's own ReLU / MaxPool branch, the
reference's fp32 run vs fp64 on its own branch; every gradient (parameters, x, t, c) and eps within 3x the reference's
error + 2e-6 relative L2."""
import pytest
import torch

from oracle import ref_cpu as R

pytestmark = pytest.mark.gpu

NF, NCF, H, B = 16, 6, 32, 2


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _rel(a, b):
    a = torch.as_tensor(a).double().cpu(); b = torch.as_tensor(b).double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-300)).item()


def _oracle(C, sd, x, t, c, sc, dtype, weight, train, kinks):
    sd = {k: (v.to(dtype) if v.is_floating_point() else v.clone()).clone() for k, v in sd.items()}
    keys = [k for k, _, kind in R.state_dict_layout(C, NF, NCF, H) if kind == "param"]
    for k in keys:
        sd[k].requires_grad_(True)
    xx, tt, cc = (v.to(dtype).clone().requires_grad_(True) for v in (x, t, c))
    with kinks:
        eps = R.unet_forward(sd, xx, tt, cc, n_feat=NF, n_cfeat=NCF, height=H, train=train,
                             shortcut=(sc[0].to(dtype), sc[1].to(dtype)))
    (eps * weight.to(dtype)).sum().backward()
    return eps.detach(), {"x": xx.grad, "t": tt.grad, "c": cc.grad, **{k: sd[k].grad for k in keys}}


def _shortcut(C):
    if C == NF:
        return torch.eye(NF).reshape(NF, NF, 1, 1), torch.zeros(NF)
    return R.draw_shortcut(C, NF)


@pytest.mark.parametrize("train", [True, False])
@pytest.mark.parametrize("C", [2, 3, 16])
@pytest.mark.parametrize("math", ["fp32", "h3"])
def test_in_channels_train_grads(C, math, train):
    """train=False: gradients through model.eval() (BatchNorm frozen on running statistics made non-trivial by one
    train forward first; they must not move)"""
    import cdm_amd
    from _kinks import Kinks, hip_kinks
    torch.manual_seed(5 + C)
    m = cdm_amd.ContextUnet(C, NF, NCF, H, conv_math=math).cuda().train()
    g = torch.Generator().manual_seed(40 + C)
    if not train:
        with torch.no_grad():
            m(torch.randn(B, C, H, H, generator=g).cuda(), torch.rand(B, generator=g).cuda(),
              torch.rand(B, NCF, generator=g).cuda())
        m.eval()
    sd = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    x = torch.randn(B, C, H, H, generator=g)
    t = torch.rand(B, generator=g)
    c = torch.rand(B, NCF, generator=g)
    weight = torch.randn(B, C, H, H, generator=g)
    xg, tg, cg = (v.cuda().requires_grad_(True) for v in (x, t, c))
    torch.manual_seed(9)
    eps = m(xg, tg, cg)
    assert eps.shape == (B, C, H, H)
    (eps * weight.cuda()).sum().backward()
    if not train:
        for k, v in m.state_dict().items():
            assert torch.equal(v.cpu(), sd[k]), k
    torch.manual_seed(9)
    sc = _shortcut(C)
    hip = {"x": xg.grad, "t": tg.grad, "c": cg.grad, **{k: p.grad for k, p in m.named_parameters()}}
    m.load_state_dict(sd)
    hk_relu, hk_pool = hip_kinks(m, x, t, c, sc, frozen=not train)
    e64h, g64h = _oracle(C, sd, x, t, c, sc, torch.float64, weight, train, Kinks(hk_relu, hk_pool))
    cap32 = Kinks()
    e32, g32 = _oracle(C, sd, x, t, c, sc, torch.float32, weight, train, cap32)
    e64r, g64r = _oracle(C, sd, x, t, c, sc, torch.float64, weight, train, Kinks(cap32.relu, cap32.pool))
    bad = []
    e_h, e_r = _rel(eps.detach(), e64h), _rel(e32, e64r)
    if e_h > 3 * e_r + 2e-6:
        bad.append(("eps", e_h, e_r))
    gmax = max(v.abs().max().item() for v in g64h.values())
    for k, ref in g64h.items():
        got = hip[k]
        assert got is not None and tuple(got.shape) == tuple(ref.shape), k
        if train and (".conv1.0.bias" in k or ".conv2.0.bias" in k):   # BN-fed conv bias: analytic gradient 0 (batch BN)
            if got.abs().max().item() > 1e-4 * gmax:
                bad.append((k, got.abs().max().item(), 0.0))
            continue
        eh, er = _rel(got, ref), _rel(g32[k], g64r[k])
        if eh > 3 * er + 2e-6:
            bad.append((k, eh, er))
    assert not bad, bad


@pytest.mark.parametrize("C", [3, 16])
@pytest.mark.parametrize("math", ["fp32", "h3"])
def test_in_channels_eval_forward(C, math):
    """no-grad eval forward (BatchNorm folded into the packed weights) vs the oracle's eval forward; running statistics
    made non-trivial by one train forward first and unchanged by the eval call"""
    import cdm_amd
    torch.manual_seed(7 + C)
    m = cdm_amd.ContextUnet(C, NF, NCF, H, conv_math=math).cuda().train()
    g = torch.Generator().manual_seed(50 + C)
    with torch.no_grad():
        m(torch.randn(B, C, H, H, generator=g).cuda(), torch.rand(B, generator=g).cuda(),
          torch.rand(B, NCF, generator=g).cuda())
    m.eval()
    sd = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    x = torch.randn(B, C, H, H, generator=g)
    t = torch.rand(B, generator=g)
    c = torch.rand(B, NCF, generator=g)
    torch.manual_seed(11)
    with torch.no_grad():
        eps = m(x.cuda(), t.cuda(), c.cuda()).cpu()
    for k, v in m.state_dict().items():
        assert torch.equal(v.cpu(), sd[k]), k
    torch.manual_seed(11)
    sc = _shortcut(C)
    ref = R.unet_forward({k: v.double() if v.is_floating_point() else v for k, v in sd.items()}, x.double(), t.double(),
                         c.double(), n_feat=NF, n_cfeat=NCF, height=H, train=False,
                         shortcut=(sc[0].double(), sc[1].double()))
    assert eps.shape == (B, C, H, H)
    assert _rel(eps, ref) < 2e-4


@pytest.mark.parametrize("C", [1, 3])
def test_device_shortcut_draw_range(C):
    """shortcut_source="device": the fresh 1x1 shortcut's weight and bias come from U(-1/sqrt(C), 1/sqrt(C)), the
    distribution of the reference's nn.Conv2d(C, n_feat, 1) init (kaiming_uniform_(a = sqrt(5)) and its bias bound,
    fan_in = C; diffusion_utilities.py:54).  ADVICE r5: the device draw was U(-1, 1) for every C."""
    import cdm_amd
    m = cdm_amd.ContextUnet(C, 128, NCF, H, shortcut_source="device").cuda()
    bound = 1.0 / C ** 0.5
    ws, bs = [], []
    for _ in range(8):
        w, b = m.draw_shortcut(torch.device("cuda"))
        assert w.numel() == 128 * C and b.numel() == 128
        ws.append(w.cpu()); bs.append(b.cpu())
    w, b = torch.cat(ws), torch.cat(bs)
    for v in (w, b):
        assert v.abs().max().item() <= bound
        assert v.abs().max().item() >= 0.95 * bound          # 1024+ draws reach the edge of the interval
        assert abs(v.mean().item()) <= 0.1 * bound and abs(v.std().item() - bound / 3 ** 0.5) <= 0.1 * bound


@pytest.mark.parametrize("C", [1, 3])
def test_in_channels_bf16_c4_arithmetic(C):
    """C4's bf16 arithmetic with in_channels = 3 at n_feat = 128 (the cp > 1 image through the bf16 matrix
    cores — the batched bf16 repack of the init conv, the fused BN / fused eval-epilogue paths, which need C_out % 128 ==
    0): eval and train forward, and every gradient (parameters, x, t, c) of a train-mode call, vs fp64, within 1.5x the
    error of the reference under C4's bf16 operand rounding (tests/_bf16emu.py; train: conv outputs / gradients stored
    in bf16 as autocast does), the bar of tests/test_gpu_configs.py's C4 tests (max and median over tensors); dL/dt, one
    heavily cancelling scalar per image, against the emulated reference's per-term error sum (below).  C = 1 alongside
    (the dedicated single-channel kernels under bf16)."""
    import numpy as np
    import cdm_amd
    from _bf16emu import _bf16_operands
    nf, Hh, Bb = 128, 32, 2
    torch.manual_seed(17)
    m = cdm_amd.ContextUnet(C, nf, NCF, Hh, conv_math="bf16").cuda()
    sd = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    g = torch.Generator().manual_seed(71)
    x = torch.randn(Bb, C, Hh, Hh, generator=g); t = torch.rand(Bb, generator=g); c = torch.rand(Bb, NCF, generator=g)
    weight = torch.randn(Bb, C, Hh, Hh, generator=g)
    sc = None

    def oracle(dtype, emulate, train):
        """(eps, gradients, dL/dt term vectors): dL/dt_b = sum_j dL/dtemb[b, j] * dtemb[b, j]/dt_b over both time
        embeddings (their outputs' gradients kept by a hook on the oracle's embed, the derivatives by forward-mode AD)"""
        s = {k: (v.to(dtype) if v.is_floating_point() else v.clone()).clone() for k, v in sd.items()}
        keys = [k for k, _, kind in R.state_dict_layout(C, nf, NCF, Hh) if kind == "param"]
        for k in keys:
            s[k].requires_grad_(True)
        xx, tt, cc = (v.to(dtype).clone().requires_grad_(True) for v in (x, t, c))
        args = dict(n_feat=nf, n_cfeat=NCF, height=Hh, train=train, shortcut=(sc[0].to(dtype), sc[1].to(dtype)))
        kept, orig = {}, R._Ctx.embed

        def embed(self, v, name, in_dim):
            out = orig(self, v, name, in_dim)
            if name.startswith("timeembed") and out.requires_grad:
                out.retain_grad()
                kept[name] = out
            return out
        R._Ctx.embed = embed
        try:
            if emulate:
                with _bf16_operands(outputs=train):
                    eps = R.unet_forward(s, xx, tt, cc, **args)
                    (eps * weight.to(dtype)).sum().backward()
            else:
                eps = R.unet_forward(s, xx, tt, cc, **args)
                (eps * weight.to(dtype)).sum().backward()
        finally:
            R._Ctx.embed = orig
        terms = []
        for name, out in kept.items():
            ctx = R._Ctx({k: v.detach() for k, v in s.items()}, False)
            _, jac = torch.func.jvp(lambda u: ctx.embed(u, name, 1), (tt.detach(),), (torch.ones_like(tt),))
            terms.append(out.grad.reshape(Bb, -1) * jac.reshape(Bb, -1))
        return eps.detach(), {"x": xx.grad, "t": tt.grad, "c": cc.grad, **{k: s[k].grad for k in keys}}, \
            torch.cat(terms, 1).double()

    res = {}
    for train in (False, True):
        m.load_state_dict(sd)
        m.train(train)
        # the module draws its shortcut from the CPU RNG (shortcut_source="cpu"): the oracle replays that draw
        torch.manual_seed(99)
        sc = R.draw_shortcut(C, nf)
        torch.manual_seed(99)
        if train:
            xg, tg, cg = (v.cuda().requires_grad_(True) for v in (x, t, c))
            eps = m(xg, tg, cg)
            (eps * weight.cuda()).sum().backward()
            hip = {"x": xg.grad, "t": tg.grad, "c": cg.grad, **{k: p.grad for k, p in m.named_parameters()}}
        else:
            with torch.no_grad():
                eps = m(x.cuda(), t.cuda(), c.cuda())
        e64, g64, t64 = oracle(torch.float64, False, train)
        ee, ge, te = oracle(torch.float32, True, train)
        res[f"eps_{'train' if train else 'eval'}"] = (_rel(eps.detach(), e64), _rel(ee, e64))
        if train:
            per = {}
            for k, ref in g64.items():
                if ".conv1.0.bias" in k or ".conv2.0.bias" in k or k == "t":
                    continue
                per[k] = (_rel(hip[k], ref), _rel(ge[k], ref))
            # dL/dt: one scalar per image, a sum of 3 n_feat terms (assert_terms_sum: it equals the fp64 gradient)
            # that cancel heavily; under bf16 gradient storage both HIP's and the emulated reference's values are
            # noise-dominated (round 6, C = 3: relative error 2.0 vs 0.39 at C = 3, 0.19 vs 0.36 at C = 1).  Bar: HIP's
            # error per image within 1.5x the largest error the emulated reference's per-term errors can add up to
            assert torch.allclose(t64.sum(1), g64["t"].double(), rtol=1e-9, atol=1e-12)
            dt_err = (hip["t"].cpu().double() - g64["t"].double()).abs()
            dt_bound = (te - t64).abs().sum(1)
            res["t_err_over_bound"] = (float((dt_err / dt_bound).max()), 1.0)
            print("dL/dt |HIP - fp64|", dt_err.tolist(), "emulated per-term error sum", dt_bound.tolist(),
                  "fp64 sum of |terms|", t64.abs().sum(1).tolist())
            gh, gm = [v[0] for v in per.values()], [v[1] for v in per.values()]
            res["grad_max"] = (max(gh), max(gm))
            res["grad_median"] = (float(np.median(gh)), float(np.median(gm)))
            print("worst tensors (HIP, emulated):", sorted(per.items(), key=lambda kv: -kv[1][0])[:6])
            print("dL/dt HIP", hip["t"].cpu().tolist(), "fp64", g64["t"].tolist(), "emulated", ge["t"].tolist())
    print(f"in_channels={C} bf16 (HIP, bf16-emulated reference):", res)
    for k, (h, e) in res.items():
        assert h <= 1.5 * e, (k, h, e)


def test_in_channels_single_channel_loops_raise():
    """the training loop and samplers (reference: in_channels = 1, [n, 1, H, W] draws) refuse other channel counts"""
    import cdm_amd
    m = cdm_amd.ContextUnet(3, NF, NCF, H).cuda()
    with pytest.raises(NotImplementedError):
        cdm_amd.DDPM(m, 10, "cuda").sample_ddpm(2, H, "cuda", torch.zeros(2, NCF).cuda(), 0.0)
