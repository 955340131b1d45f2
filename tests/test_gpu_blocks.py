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


def test_embed_fc_forward_and_no_backward():
    from cdm_amd import EmbedFC
    torch.manual_seed(4)
    cpu = EmbedFC(6, 64)
    gpu = copy.deepcopy(cpu).cuda()
    x = torch.rand(5, 6)
    with torch.no_grad():
        ref = cpu.model(x.view(-1, 6))
    got = gpu(x.cuda())
    assert _rel(got, ref) < 1e-5
    with pytest.raises(NotImplementedError):
        got.sum().backward()
