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


def test_in_channels_single_channel_loops_raise():
    """the training loop and samplers (reference: in_channels = 1, [n, 1, H, W] draws) refuse other channel counts"""
    import cdm_amd
    m = cdm_amd.ContextUnet(3, NF, NCF, H).cuda()
    with pytest.raises(NotImplementedError):
        cdm_amd.DDPM(m, 10, "cuda").sample_ddpm(2, H, "cuda", torch.zeros(2, NCF).cuda(), 0.0)
