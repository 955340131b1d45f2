"""Standalone block forwards (cdm_amd.blocks) vs the reference's block semantics run by torch on the CPU in fp32
(diffusion_utilities.py:39-65, 94-100, 114-116, 137-145): train mode (batch statistics, running statistics updated) and
eval mode.  Tolerance: max |d| <= 1e-4 max |ref| (the fp32 bar of tests/test_gpu_model.py)."""
import copy

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _rcb_ref(blk, x):   # ResidualConvBlock.forward of the reference, on CPU torch modules (is_res False)
    return blk.conv2(blk.conv1(x))


def _rel(a, b):
    return (a.detach().cpu() - b.detach()).abs().max().item() / b.detach().abs().max().item()


def _pair(mod):
    torch.manual_seed(0)
    return mod, copy.deepcopy(mod).cuda()


@pytest.mark.parametrize("train", [True, False])
def test_residual_block_forward(train):
    from cdm_amd import ResidualConvBlock
    torch.manual_seed(1)
    cpu = ResidualConvBlock(16, 32)
    for bn in (cpu.conv1[1], cpu.conv2[1]):
        bn.running_mean.uniform_(-0.1, 0.1); bn.running_var.uniform_(0.5, 1.5)
    gpu = copy.deepcopy(cpu).cuda()
    cpu.train(train); gpu.train(train)
    x = torch.randn(3, 16, 16, 16)
    with torch.no_grad():
        ref = _rcb_ref(cpu, x)
        got = gpu(x.cuda())
    assert _rel(got, ref) < 1e-4, _rel(got, ref)
    for k, v in cpu.state_dict().items():
        assert torch.allclose(gpu.state_dict()[k].cpu().float(), v.float(), rtol=1e-5, atol=1e-6), k


def test_residual_block_is_res_shortcut_replays_cpu_rng():
    """init_conv form: is_res with in_channels = 1, a fresh 1x1 shortcut drawn from the CPU RNG per call."""
    from cdm_amd import ResidualConvBlock
    torch.manual_seed(2)
    cpu = ResidualConvBlock(1, 32, is_res=True)
    gpu = copy.deepcopy(cpu).cuda()
    x = torch.randn(2, 1, 16, 16)
    torch.manual_seed(7)
    with torch.no_grad():
        x2 = _rcb_ref(cpu, x)
        ref = torch.nn.Conv2d(1, 32, 1)(x) + x2
    torch.manual_seed(7)
    with torch.no_grad():
        got = gpu(x.cuda())
    assert _rel(got, ref) < 1e-4


def test_unet_down_and_up_forward():
    from cdm_amd import UnetDown, UnetUp
    torch.manual_seed(3)
    down, up = UnetDown(16, 32), UnetUp(64, 32)
    gd, gu = copy.deepcopy(down).cuda(), copy.deepcopy(up).cuda()
    x = torch.randn(2, 16, 16, 16)
    skip = torch.randn(2, 32, 8, 8)
    with torch.no_grad():
        rd = F.max_pool2d(_rcb_ref(down.model[1], _rcb_ref(down.model[0], x)), 2)
        ru = _rcb_ref(up.model[2], _rcb_ref(up.model[1], up.model[0](torch.cat((rd, skip), 1))))
        got_d = gd(x.cuda())
        got_u = gu(got_d, skip.cuda())
    assert _rel(got_d, rd) < 1e-4
    assert _rel(got_u, ru) < 1e-4


def test_embed_fc_forward():
    from cdm_amd import EmbedFC
    torch.manual_seed(4)
    cpu = EmbedFC(6, 64)
    gpu = copy.deepcopy(cpu).cuda()
    x = torch.rand(5, 6)
    with torch.no_grad():
        ref = cpu.model(x.view(-1, 6))
    got = gpu(x.cuda())
    assert _rel(got, ref) < 1e-5


# ---------------------------------------------------------------------------------------------- backward (train mode)
# The standalone blocks' backward (the tape replay on the HIP kernels) vs torch autograd of the reference block
# semantics on the CPU in fp32: every parameter gradient and the input gradient(s), relative L2 <= 1e-4 (BatchNorm with
# batch statistics amplifies summation-order noise, as in tests/test_gpu_model.py); the conv biases that feed a
# BatchNorm have analytic gradient 0 on both sides (|g| <= 1e-5 max over all gradients).

def _grad_check(cpu_mod, gpu_mod, ref_fn, got_fn, inputs, seed=9):
    g = torch.Generator().manual_seed(seed)
    xs_c = [x.clone().requires_grad_(True) for x in inputs]
    out = ref_fn(*xs_c)
    w = torch.randn(out.shape, generator=g)
    (out * w).sum().backward()
    xs_g = [x.cuda().requires_grad_(True) for x in inputs]
    got = got_fn(*xs_g)
    assert _rel(got, out) < 1e-4
    (got * w.cuda()).sum().backward()
    ref = dict(cpu_mod.named_parameters())
    gmax = max(p.grad.abs().max().item() for p in ref.values())
    for n, p in gpu_mod.named_parameters():
        r = ref[n].grad
        assert p.grad is not None, n
        if n.endswith("0.bias") and ("conv1" in n or "conv2" in n):
            assert p.grad.abs().max().item() <= 1e-5 * gmax, n
            continue
        e = ((p.grad.cpu() - r).norm() / r.norm()).item()
        assert e < 1e-4, (n, e)
    for xc, xg in zip(xs_c, xs_g):
        e = ((xg.grad.cpu() - xc.grad).norm() / xc.grad.norm()).item()
        assert e < 1e-4, e


def test_residual_block_backward():
    from cdm_amd import ResidualConvBlock
    torch.manual_seed(11)
    cpu = ResidualConvBlock(16, 32)
    gpu = copy.deepcopy(cpu).cuda()
    cpu.train(); gpu.train()
    _grad_check(cpu, gpu, lambda x: _rcb_ref(cpu, x), gpu, [torch.randn(3, 16, 16, 16)])


def test_residual_block_is_res_backward_params():
    """init_conv form (is_res, C_in = 1, the fresh CPU-RNG 1x1 shortcut): parameter gradients (the image needs none;
    its gradient is not built on the HIP path and raises when asked for)."""
    from cdm_amd import ResidualConvBlock
    torch.manual_seed(12)
    cpu = ResidualConvBlock(1, 32, is_res=True)
    gpu = copy.deepcopy(cpu).cuda()
    x = torch.randn(2, 1, 16, 16)
    g = torch.randn(2, 32, 16, 16)
    torch.manual_seed(7)
    ref = torch.nn.Conv2d(1, 32, 1)(x).detach() + _rcb_ref(cpu, x)
    (ref * g).sum().backward()
    torch.manual_seed(7)
    got = gpu(x.cuda())
    assert _rel(got, ref) < 1e-4
    (got * g.cuda()).sum().backward()
    refp = dict(cpu.named_parameters())
    for n, p in gpu.named_parameters():
        if n.endswith("0.bias"):
            continue
        e = ((p.grad.cpu() - refp[n].grad).norm() / refp[n].grad.norm()).item()
        assert e < 1e-4, (n, e)


@pytest.mark.parametrize("is_res", [True, False])
def test_residual_block_cin1_image_grad(is_res):
    """The image gradient of a C_in = 1 block (ContextUnet's init_conv form): the tap-flipped conv over conv1's BN
    backward plus, for is_res, the fresh 1x1 shortcut's sum_c w[c] g[c]; vs torch autograd on the CPU."""
    from cdm_amd import ResidualConvBlock
    torch.manual_seed(3)
    cpu = ResidualConvBlock(1, 32, is_res=is_res)
    gpu = copy.deepcopy(cpu).cuda()
    g_ = torch.Generator().manual_seed(4)
    x = torch.randn(2, 1, 16, 16, generator=g_)
    w = torch.randn(2, 32, 16, 16, generator=g_)
    xc = x.clone().requires_grad_(True)
    torch.manual_seed(7)
    ref = (torch.nn.Conv2d(1, 32, 1)(xc) + _rcb_ref(cpu, xc)) if is_res else _rcb_ref(cpu, xc)
    (ref * w).sum().backward()
    xg = x.cuda().requires_grad_(True)
    torch.manual_seed(7)
    got = gpu(xg)
    assert _rel(got, ref) < 1e-4
    (got * w.cuda()).sum().backward()
    e = ((xg.grad.cpu() - xc.grad).norm() / xc.grad.norm()).item()
    assert e < 1e-4, e


def test_unet_down_up_backward():
    from cdm_amd import UnetDown, UnetUp
    torch.manual_seed(13)
    down, up = UnetDown(16, 32), UnetUp(64, 32)
    gd, gu = copy.deepcopy(down).cuda(), copy.deepcopy(up).cuda()
    _grad_check(down, gd, lambda x: F.max_pool2d(_rcb_ref(down.model[1], _rcb_ref(down.model[0], x)), 2), gd,
                [torch.randn(2, 16, 16, 16)])

    def ref_up(x, skip):
        return _rcb_ref(up.model[2], _rcb_ref(up.model[1], up.model[0](torch.cat((x, skip), 1))))
    _grad_check(up, gu, ref_up, gu, [torch.randn(2, 32, 8, 8), torch.randn(2, 32, 8, 8)])


@pytest.mark.parametrize("in_dim", [1, 5, 6, 8])
def test_embed_fc_backward(in_dim):
    """EmbedFC alone, parameter and input gradients for every input_dim (the reference's t embedding takes 1, its
    context embeddings n_cfeat = 5 or 6: diffusion_utilities.py:118-145, ContextUnet.py:22-23)."""
    from cdm_amd import EmbedFC
    torch.manual_seed(14)
    cpu = EmbedFC(in_dim, 64)
    gpu = copy.deepcopy(cpu).cuda()
    x = torch.rand(5, in_dim)
    _grad_check(cpu, gpu, lambda v: cpu.model(v.view(-1, in_dim)), gpu, [x])


@pytest.mark.parametrize("kind", ["rcb", "down", "cin1_res"])
def test_eval_block_backward(kind):
    """Gradients through an eval-mode block (BatchNorm on the running statistics, batch_norm(training=False) under
    autograd: the conv biases get a gradient here), parameters and input, vs torch autograd of the same modules in eval
    mode on the CPU; running statistics untouched."""
    from cdm_amd import ResidualConvBlock, UnetDown
    torch.manual_seed(17)
    if kind == "rcb":
        cpu, shape = ResidualConvBlock(16, 32), (2, 16, 8, 8)
        ref_fn = lambda v: _rcb_ref(cpu, v)   # noqa: E731
    elif kind == "down":
        cpu, shape = UnetDown(16, 32), (2, 16, 16, 16)
        ref_fn = lambda v: F.max_pool2d(_rcb_ref(cpu.model[1], _rcb_ref(cpu.model[0], v)), 2)   # noqa: E731
    else:
        cpu, shape = ResidualConvBlock(1, 32, is_res=True), (2, 1, 16, 16)
        ref_fn = lambda v: torch.nn.Conv2d(1, 32, 1)(v) + _rcb_ref(cpu, v)   # noqa: E731
    for m in cpu.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.running_mean.uniform_(-0.2, 0.2); m.running_var.uniform_(0.5, 1.5)
    cpu.eval()
    gpu = copy.deepcopy(cpu).cuda().eval()
    run0 = {k: v.clone() for k, v in gpu.state_dict().items()}
    g_ = torch.Generator().manual_seed(18)
    x = torch.randn(*shape, generator=g_)
    xc = x.clone().requires_grad_(True)
    torch.manual_seed(7)
    ref = ref_fn(xc)
    w = torch.randn(ref.shape, generator=g_)
    (ref * w).sum().backward()
    xg = x.cuda().requires_grad_(True)
    torch.manual_seed(7)
    got = gpu(xg)
    assert _rel(got, ref) < 1e-4
    (got * w.cuda()).sum().backward()
    refp = dict(cpu.named_parameters())
    for n, p in gpu.named_parameters():
        r = refp[n].grad
        assert p.grad is not None, n
        e = ((p.grad.cpu() - r).norm() / r.norm()).item()
        assert e < 1e-4, (n, e)
    e = ((xg.grad.cpu() - xc.grad).norm() / xc.grad.norm()).item()
    assert e < 1e-4, e
    for k, v in gpu.state_dict().items():
        assert torch.equal(v, run0[k]), k


@pytest.mark.parametrize("cin,cout", [(32, 32), (16, 32)])
def test_residual_block_is_res_same_and_wide(cin, cout):
    """is_res blocks beyond ContextUnet's C_in = 1 form (diffusion_utilities.py:39-65): same channels out = x + x2,
    wider out = shortcut(x) + x2 with the fresh CPU-RNG 1x1 shortcut of every call; forward and the train-mode backward
    (parameters and input) vs torch autograd on the CPU."""
    from cdm_amd import ResidualConvBlock
    torch.manual_seed(15)
    cpu = ResidualConvBlock(cin, cout, is_res=True)
    gpu = copy.deepcopy(cpu).cuda()
    g = torch.Generator().manual_seed(16)
    x = torch.randn(2, cin, 16, 16, generator=g)
    w = torch.randn(2, cout, 16, 16, generator=g)
    xc = x.clone().requires_grad_(True)
    torch.manual_seed(7)
    x2 = _rcb_ref(cpu, xc)
    ref = xc + x2 if cin == cout else torch.nn.Conv2d(cin, cout, 1)(xc) + x2
    (ref * w).sum().backward()
    xg = x.cuda().requires_grad_(True)
    torch.manual_seed(7)
    got = gpu(xg)
    assert _rel(got, ref) < 1e-4
    (got * w.cuda()).sum().backward()
    refp = dict(cpu.named_parameters())
    for n, p in gpu.named_parameters():
        if n.endswith("0.bias"):
            continue
        e = ((p.grad.cpu() - refp[n].grad).norm() / refp[n].grad.norm()).item()
        assert e < 1e-4, (n, e)
    e = ((xg.grad.cpu() - xc.grad).norm() / xc.grad.norm()).item()
    assert e < 1e-4, e
