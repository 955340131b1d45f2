"""Standalone forwards of the reference's building blocks on the HIP kernels (diffusion_utilities.py:39-65 ResidualConvBlock,
:94-100 UnetUp, :114-116 UnetDown, :137-145 EmbedFC).

Inside ContextUnet the blocks never run one by one (the engine executes the network as a whole, with its fused
layouts); these forwards serve code that calls a block on its own.  They run the same kernels the engine uses — 3x3
convs in plain fp32 MFMA (`cdm_conv3x3_fwd`), BatchNorm statistics from the conv epilogue folded in fp64 (train mode,
running statistics updated like torch) or folded into the packed weights (eval), fused ReLU / MaxPool / shortcut
applies, the 2x2 ConvTranspose GEMM, the EmbedFC kernel — on NHWC copies of the NCHW inputs.  Forward only: the
result carries an autograd node whose backward raises (training runs through ContextUnet / Trainer).
"""
from __future__ import annotations

import ctypes
import types

import torch
import torch.nn as nn

from ._lib import Mlp4, lib
from .engine import APPLY_POOL, APPLY_RELU, APPLY_RESID, CHUNK, EPI_RELU, _cdiv, conv_kc, fold


def _p(t):
    return None if t is None else t.data_ptr()


def _s() -> int:
    return torch.cuda.current_stream().cuda_stream


class _BlockNoBackward(torch.autograd.Function):
    @staticmethod
    def forward(ctx, out, *params):
        return out.view_as(out)

    @staticmethod
    def backward(ctx, *grads):
        raise NotImplementedError("standalone block forwards on the HIP engine are forward-only; differentiate through "
                                  "ContextUnet (or cdm_amd.Trainer)")


def _finish(out: torch.Tensor, module: nn.Module) -> torch.Tensor:
    params = [p for p in module.parameters() if p.requires_grad]
    if torch.is_grad_enabled() and params:
        return _BlockNoBackward.apply(out, *params)
    return out


def _check(x: torch.Tensor, what: str):
    if x.device.type != "cuda":
        raise RuntimeError(f"{what} runs on the MI355X HIP kernels: move the module and its input to a cuda device")
    return x.detach().to(torch.float32).contiguous()


def to_nhwc(x: torch.Tensor) -> torch.Tensor:
    """[B, C, H, W] -> [B*H*W, C] (cdm_transpose_batched)."""
    B, C, H, W = x.shape
    out = torch.empty(B * H * W, C, device=x.device)
    lib().cdm_transpose_batched(x.data_ptr(), B, C, H * W, out.data_ptr(), _s())
    return out


def to_nchw(y: torch.Tensor, B: int, H: int, W: int, C: int) -> torch.Tensor:
    out = torch.empty(B, C, H, W, device=y.device)
    lib().cdm_transpose_batched(y.data_ptr(), B, H * W, C, out.data_ptr(), _s())
    return out


def conv_bn_relu(seq: nn.Sequential, xh: torch.Tensor, B: int, H: int, W: int, pool: bool = False, resid=None):
    """Conv2d(3x3) -> BatchNorm2d -> ReLU (diffusion_utilities.py:26-37) on NHWC xh [B*H*W, Cin]; optionally the
    MaxPool2d(2) after it (UnetDown) or the reference's C_in = 1 shortcut add (resid = (x [B*H*W], w [C], b [C]))."""
    L, s = lib(), _s()
    conv, bn = seq[0], seq[1]
    Cin, Cout = conv.in_channels, conv.out_channels
    if Cout % 4:
        raise NotImplementedError("the HIP conv path needs out_channels % 4 == 0")
    dev = xh.device
    P = B * H * W
    kc = conv_kc(Cin, Cout)
    E = lambda *shape: torch.empty(*shape, device=dev)   # noqa: E731
    Wt, bt = conv.weight.detach().contiguous(), conv.bias.detach().contiguous()
    if bn.training:
        wpk = E(9 * Cin, Cout)
        L.cdm_pack_conv3x3(Wt.data_ptr(), bt.data_ptr(), Cin, Cout, None, None, None, None, 0.0, wpk.data_ptr(), None,
                           None, kc, s)
        y = E(P, Cout)
        if Cin == 1:
            L.cdm_conv3x3_cin1_fwd(xh.data_ptr(), B, H, W, wpk.data_ptr(), bt.data_ptr(), y.data_ptr(), Cout, Cout, 0,
                                   None, s)
            ntiles = B * _cdiv(H * W, CHUNK)
            slab = E(ntiles * 2 * Cout)
            L.cdm_reduce_stats(y.data_ptr(), Cout, B, H * W, Cout, CHUNK, slab.data_ptr(), s)
        else:
            ntiles = _cdiv(P, CHUNK)
            slab = E(ntiles * 2 * Cout)
            L.cdm_conv3x3_fwd(xh.data_ptr(), B, H, W, Cin, Cin, wpk.data_ptr(), bt.data_ptr(), y.data_ptr(), Cout, Cout,
                              0, slab.data_ptr(), Cout, kc, s)
        ws = types.SimpleNamespace(dpart=torch.empty(10 * 32768 + 4096, device=dev, dtype=torch.float64))
        nparts = fold(ws, slab.data_ptr(), ntiles, 2, Cout, s)
        st = [E(Cout) for _ in range(4)]                  # mean, invstd, scale, shift
        track = bn.track_running_stats and bn.running_mean is not None
        mom = 0.1 if bn.momentum is None else float(bn.momentum)
        L.cdm_bn_fwd_finalize(ws.dpart.data_ptr(), nparts, 2, Cout, float(P), bn.weight.data_ptr(), bn.bias.data_ptr(),
                              _p(bn.running_mean) if track else None, _p(bn.running_var) if track else None,
                              _p(bn.num_batches_tracked) if track else None, mom, float(bn.eps),
                              *[t.data_ptr() for t in st], None, 0, None, s)
        scale, shift, flags = st[2], st[3], APPLY_RELU
    else:
        wpk, bpk = E(9 * Cin, Cout), E(Cout)
        L.cdm_pack_conv3x3(Wt.data_ptr(), bt.data_ptr(), Cin, Cout, bn.weight.data_ptr(), bn.bias.data_ptr(),
                           bn.running_mean.data_ptr(), bn.running_var.data_ptr(), float(bn.eps), wpk.data_ptr(),
                           bpk.data_ptr(), None, kc, s)
        y = E(P, Cout)
        if Cin == 1:
            L.cdm_conv3x3_cin1_fwd(xh.data_ptr(), B, H, W, wpk.data_ptr(), bpk.data_ptr(), y.data_ptr(), Cout, Cout, 1,
                                   None, s)
        else:
            L.cdm_conv3x3_fwd(xh.data_ptr(), B, H, W, Cin, Cin, wpk.data_ptr(), bpk.data_ptr(), y.data_ptr(), Cout,
                              Cout, EPI_RELU, None, 0, kc, s)
        if not pool and resid is None:
            return y
        scale, shift, flags = torch.ones(Cout, device=dev), torch.zeros(Cout, device=dev), 0
    if pool:
        out = E(B * (H // 2) * (W // 2), Cout)
        L.cdm_norm_apply_fwd(APPLY_POOL | flags, y.data_ptr(), Cout, B, H, W, Cout, scale.data_ptr(), shift.data_ptr(), 0,
                             None, 0, None, 0, None, None, None, 0, out.data_ptr(), Cout, None, s)
        return out
    out = E(P, Cout)
    rx, rw, rb = resid if resid is not None else (None, None, None)
    L.cdm_norm_apply_fwd((APPLY_RESID if resid is not None else 0) | flags, y.data_ptr(), Cout, B, H, W, Cout,
                         scale.data_ptr(), shift.data_ptr(), 0, None, 0, None, 0, _p(rx), _p(rw), _p(rb), B,
                         out.data_ptr(), Cout, None, s)
    return out


def residual_block(blk, xh: torch.Tensor, x_nchw: torch.Tensor, B: int, H: int, W: int, pool: bool = False):
    """ResidualConvBlock.forward (diffusion_utilities.py:39-65) on NHWC xh."""
    resid = None
    if blk.is_res:
        Cin, Cout = blk.conv1[0].in_channels, blk.conv2[0].out_channels
        if blk.same_channels or Cin != 1:
            raise NotImplementedError("the HIP block path implements the reference's is_res shortcut for in_channels=1 "
                                      "(ContextUnet's init_conv); same-channel / wider residual adds are not built")
        # the reference draws a fresh 1x1 conv on every call (diffusion_utilities.py:54): same CPU RNG consumption
        sc = nn.Conv2d(Cin, Cout, kernel_size=1, stride=1, padding=0)
        resid = (x_nchw.reshape(-1).contiguous(), sc.weight.detach().reshape(Cout).to(xh.device),
                 sc.bias.detach().to(xh.device))
    z1 = conv_bn_relu(blk.conv1, xh, B, H, W)
    return conv_bn_relu(blk.conv2, z1, B, H, W, pool=pool, resid=resid)


def residual_block_forward(blk, x: torch.Tensor) -> torch.Tensor:
    x = _check(x, "ResidualConvBlock")
    B, _, H, W = x.shape
    y = residual_block(blk, to_nhwc(x), x, B, H, W)
    return _finish(to_nchw(y, B, H, W, blk.conv2[0].out_channels), blk)


def unet_down_forward(mod, x: torch.Tensor) -> torch.Tensor:
    """UnetDown.forward (diffusion_utilities.py:114-116): 2 ResidualConvBlocks + MaxPool2d(2)."""
    x = _check(x, "UnetDown")
    B, _, H, W = x.shape
    if H % 2 or W % 2:
        raise NotImplementedError("the fused MaxPool2d(2) needs even H and W")
    z = residual_block(mod.model[0], to_nhwc(x), x, B, H, W)
    z = residual_block(mod.model[1], z, None, B, H, W, pool=True)
    return _finish(to_nchw(z, B, H // 2, W // 2, mod.model[1].conv2[0].out_channels), mod)


def unet_up_forward(mod, x: torch.Tensor, skip: torch.Tensor) -> torch.Tensor:
    """UnetUp.forward (diffusion_utilities.py:94-100): cat(x, skip) -> ConvTranspose2d(2, 2) -> 2 ResidualConvBlocks."""
    x = _check(torch.cat((x, skip), 1), "UnetUp")
    L, s = lib(), _s()
    B, Cin, H, W = x.shape
    ct = mod.model[0]
    Cout = ct.out_channels
    if Cin % 4 or Cout % 4:
        raise NotImplementedError("the HIP ConvTranspose path needs channels % 4 == 0")
    wt = torch.empty(Cin, 4 * Cout, device=x.device)
    L.cdm_pack_convT(ct.weight.detach().contiguous().data_ptr(), Cin, Cout, 4, wt.data_ptr(), None, s)
    y = torch.empty(B * 4 * H * W, Cout, device=x.device)
    L.cdm_convT2x2_fwd(to_nhwc(x).data_ptr(), B, H, W, Cin, Cin, wt.data_ptr(), ct.bias.detach().data_ptr(), y.data_ptr(),
                       Cout, Cout, None, s)
    z = residual_block(mod.model[1], y, None, B, 2 * H, 2 * W)
    z = residual_block(mod.model[2], z, None, B, 2 * H, 2 * W)
    return _finish(to_nchw(z, B, 2 * H, 2 * W, mod.model[2].conv2[0].out_channels), mod)


def embed_fc_forward(mod, x: torch.Tensor) -> torch.Tensor:
    """EmbedFC.forward (diffusion_utilities.py:137-145): x.view(-1, input_dim) -> Linear -> GELU -> Linear."""
    dev = next(mod.parameters()).device
    x = _check(x.to(dev), "EmbedFC").reshape(-1, mod.input_dim).contiguous()
    l1, l2 = mod.model[0], mod.model[2]
    E = l1.out_features
    if E > 1024:
        raise NotImplementedError("the EmbedFC kernel holds the hidden vector in LDS: emb_dim <= 1024")
    rows = x.shape[0]
    w2 = l2.weight.detach().contiguous()
    w2t = torch.empty(E, E, device=dev)
    lib().cdm_transpose(w2.data_ptr(), E, E, w2t.data_ptr(), _s())
    out = torch.empty(rows, E, device=dev)
    d = Mlp4()
    m = d.m[0]
    m.x, m.rows, m.in_dim, m.E = x.data_ptr(), rows, mod.input_dim, E
    m.w1, m.b1 = l1.weight.detach().contiguous().data_ptr(), l1.bias.detach().data_ptr()
    m.w2, m.w2t, m.b2 = w2.data_ptr(), w2t.data_ptr(), l2.bias.detach().data_ptr()
    m.out = out.data_ptr()
    for k in (1, 2, 3):
        d.m[k].rows = 0
    lib().cdm_embed_fwd(ctypes.addressof(d), _s())  # the descriptor is copied into the launch's kernel arguments
    return _finish(out, mod)
