"""Standalone forwards of the reference's building blocks on the HIP kernels (diffusion_utilities.py:39-65 ResidualConvBlock,
:94-100 UnetUp, :114-116 UnetDown, :137-145 EmbedFC).

Inside ContextUnet the blocks never run one by one (the engine executes the network as a whole, with its fused
layouts); these forwards serve code that calls a block on its own.  They run the same kernels the engine uses — 3x3
convs in plain fp32 MFMA (`cdm_conv3x3_fwd`), BatchNorm statistics from the conv epilogue folded in fp64 (train mode,
running statistics updated like torch) or folded into the packed weights (eval), fused ReLU / MaxPool / shortcut
applies, the 2x2 ConvTranspose GEMM, the EmbedFC kernel — on NHWC copies of the NCHW inputs.

Train-mode calls that need gradients record a tape (per Conv -> BatchNorm -> ReLU layer: its input, pre-norm output,
batch statistics and dgrad weights; per ConvTranspose: its input and transposed weights; per EmbedFC: its hidden
pre-activation and activation) and return through one autograd node whose backward replays the tape on the HIP
kernels the engine uses for the same layers: BatchNorm / ReLU / MaxPool backward sums and apply
(`cdm_norm_bwd_reduce`, `cdm_bn_bwd_finalize`, `cdm_norm_apply_bwd`), conv weight gradients (`cdm_conv3x3_wgrad`, the
C_in = 1 form `cdm_conv3x3_cin1_wgrad`), input gradients (the conv on the flipped weights), ConvTranspose backward
(`cdm_convT2x2_wgrad / dgrad`), EmbedFC backward (`cdm_embed_bwd`).  Parameter gradients always; the input gradient
of every input (EmbedFC: any input_dim), incl. the C_in = 1 image of a ResidualConvBlock(1, C) (the flipped-weight
conv `cdm_conv3x3_cin1_dgrad`, plus the random 1x1 shortcut's sum_c w[c] g[c] for is_res).  Eval-mode calls under
autograd run the same taped form with BatchNorm frozen on the running statistics (`cdm_bn_fwd_frozen`, backward
`cdm_bn_bwd_finalize_frozen`: the backward of batch_norm(training=False)), as ContextUnet's.
"""
from __future__ import annotations

import ctypes
import types

import torch
import torch.nn as nn

from ._lib import Mlp4, lib
from .engine import APPLY_POOL, APPLY_RELU, APPLY_RESID, CHUNK, EPI_ACCUM, EPI_RELU, _cdiv, conv_kc, fold, wgrad_splits


def _p(t):
    return None if t is None else t.data_ptr()


def _s() -> int:
    return torch.cuda.current_stream().cuda_stream


def _finish(out: torch.Tensor, module: nn.Module, tape=None, inputs=()) -> torch.Tensor:
    params = [p for p in module.parameters() if p.requires_grad]
    if torch.is_grad_enabled() and (params or any(x.requires_grad for x in inputs)):
        assert tape is not None, "a differentiable block call records a tape"
        return _BlockFunction.apply(tape, out, len(inputs), *inputs, *params)
    return out


def _dpart(dev):
    return types.SimpleNamespace(dpart=torch.empty(10 * 32768 + 4096, device=dev, dtype=torch.float64))


class _Tape:
    """The train-mode records of one standalone block call, replayed backwards on the HIP kernels.  ops: a list of
    callables g -> g' (NHWC gradient of an op's output -> of its input); each writes its parameter gradients into
    self.grads (id(param) -> tensor)."""

    def __init__(self):
        self.ops = []
        self.grads = {}
        self.first_rec = None      # the block's first conv layer: its input gradient only when the input needs one
        self.need_input = True
        self.resid_g = None        # C_in = 1 is_res block: the block-output gradient and the shortcut weights, for the
        self.resid_w = None        # image gradient (sum_c w[c] g[c]) added by the first layer's backward

    def need_dx(self, rec) -> bool:
        return rec is not self.first_rec or self.need_input

    def add(self, param, g):
        if param.requires_grad:
            self.grads[id(param)] = g

    def run(self, g):
        for op in reversed(self.ops):
            g = op(g)
        return g


class _BlockFunction(torch.autograd.Function):
    """Autograd node of a standalone block call: backward = the tape (NCHW gradients in and out)."""

    @staticmethod
    def forward(ctx, tape, out, n_in, *rest):
        ctx.tape, ctx.n_in = tape, n_in
        ctx.in_shapes = [tuple(x.shape) for x in rest[:n_in]]
        ctx.in_devices = [x.device for x in rest[:n_in]]
        # the tape reads the live parameter storage at backward time (BatchNorm weights, biases, EmbedFC weights):
        # saved here so that autograd's version check raises when one was modified in place in between
        ctx.save_for_backward(*rest[n_in:])
        return out.view_as(out)

    @staticmethod
    def backward(ctx, gout):
        params = ctx.saved_tensors          # raises if a parameter was updated in place after the forward
        tape = ctx.tape
        need = list(ctx.needs_input_grad[3:3 + ctx.n_in])
        gin = tape.backward(gout.detach().to(torch.float32).contiguous(), need, ctx.in_shapes)
        gin = [None if g is None else g.to(d) for g, d in zip(gin, ctx.in_devices)]   # e.g. a CPU EmbedFC input
        pgrads = tuple(tape.grads.get(id(p)) for p in params)
        return (None, None, None) + tuple(gin) + pgrads


def _layer_backward(rec, tape: _Tape, g: torch.Tensor, need_dx: bool):
    """Conv3x3 -> BatchNorm2d (batch statistics) -> ReLU [-> MaxPool2d(2)] [+ the C_in = 1 shortcut] backward
    (diffusion_utilities.py:26-37 under autograd): g = NHWC gradient of the layer output; returns the NHWC gradient of
    its input (None when not needed)."""
    L, s = lib(), _s()
    B, H, W, Cin, Cout = rec["dims"]
    conv, bn = rec["conv"], rec["bn"]
    dev = g.device
    P = B * H * W
    E = lambda *shape: torch.empty(*shape, device=dev)   # noqa: E731
    mean, invstd, scale, shift = rec["st"]
    y = rec["y"]
    mode = 1 if rec["pool"] else 0
    HWp = (H // 2) * (W // 2) if rec["pool"] else H * W
    nch = _cdiv(HWp, CHUNK)
    slab = E(B * nch * 5 * Cout)
    L.cdm_norm_bwd_reduce(mode, g.data_ptr(), Cout, y.data_ptr(), Cout, B, H, W, Cout, scale.data_ptr(),
                          shift.data_ptr(), 0, mean.data_ptr(), invstd.data_ptr(), 0, 1, None, 0, CHUNK, slab.data_ptr(),
                          s)
    ws = _dpart(dev)
    nparts = fold(ws, slab.data_ptr(), B * nch, 5, Cout, s)
    dgamma, dbeta, A, Bc, Cc, dbias = [E(Cout) for _ in range(6)]
    fin = L.cdm_bn_bwd_finalize_frozen if rec["frozen"] else L.cdm_bn_bwd_finalize
    fin(ws.dpart.data_ptr(), nparts, Cout, float(P), bn.weight.data_ptr(), invstd.data_ptr(), dgamma.data_ptr(),
        dbeta.data_ptr(), A.data_ptr(), Bc.data_ptr(), Cc.data_ptr(), dbias.data_ptr(), s)
    if rec.get("resid_w") is not None:       # this layer's apply added the C_in = 1 shortcut: keep g for the image grad
        tape.resid_g, tape.resid_w = g, rec["resid_w"]
    dy = E(P, Cout)
    L.cdm_norm_apply_bwd(mode, g.data_ptr(), Cout, y.data_ptr(), Cout, B, H, W, Cout, scale.data_ptr(), shift.data_ptr(),
                         0, mean.data_ptr(), invstd.data_ptr(), 0, 1, None, 0, A.data_ptr(), Bc.data_ptr(), Cc.data_ptr(),
                         0, dy.data_ptr(), Cout, None, s)
    xh = rec["x"]
    dW = E(Cout, Cin, 3, 3)
    dx = None
    if Cin > 1:
        sp = wgrad_splits(P, Cout, 9 * Cin)
        slw = E(sp * Cout * 9 * Cin)
        L.cdm_conv3x3_wgrad(dy.data_ptr(), Cout, Cout, xh.data_ptr(), B, H, W, Cin, Cin, sp, slw.data_ptr(), s)
        L.cdm_slab_reduce(slw.data_ptr(), sp, Cout, 9 * Cin, dW.data_ptr(), 9 * Cin, 1, 9, Cin, 0, 1.0, s)
        if need_dx:
            dx = E(P, Cin)
            L.cdm_conv3x3_fwd(dy.data_ptr(), B, H, W, Cout, Cout, rec["wdg"].data_ptr(), None, dx.data_ptr(), Cin, Cin,
                              0, None, 0, rec["kc"], s)
    else:
        nt = B * _cdiv(H * W, CHUNK)
        slw = E(nt * 10 * Cout)
        L.cdm_conv3x3_cin1_wgrad(dy.data_ptr(), Cout, xh.data_ptr(), B, H, W, Cout, CHUNK, slw.data_ptr(), s)
        nparts = fold(ws, slw.data_ptr(), nt, 10, Cout, s)
        L.cdm_slab_sum_all(ws.dpart.data_ptr(), nparts, 10, 0, 9, Cout, dW.data_ptr(), 1, 9, 0, s)
        if need_dx:   # the image: the tap-flipped conv over dy, plus the shortcut's sum_c w[c] g_out[c] (is_res)
            dx = E(P)
            gres, sw = tape.resid_g, tape.resid_w
            L.cdm_conv3x3_cin1_dgrad(dy.data_ptr(), Cout, None, 0, None, None, None, None, None, None, None,
                                     conv.weight.detach().contiguous().data_ptr(), _p(gres), Cout if gres is not None else 0,
                                     _p(sw), B, B, H, W, Cout, dx.data_ptr(), s)
    tape.add(conv.weight, dW)
    tape.add(conv.bias, dbias)
    tape.add(bn.weight, dgamma)
    tape.add(bn.bias, dbeta)
    return dx


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


def conv_bn_relu(seq: nn.Sequential, xh: torch.Tensor, B: int, H: int, W: int, pool: bool = False, resid=None,
                 tape: "_Tape" = None):
    """Conv2d(3x3) -> BatchNorm2d -> ReLU (diffusion_utilities.py:26-37) on NHWC xh [B*H*W, Cin]; optionally the
    MaxPool2d(2) after it (UnetDown) or the reference's C_in = 1 shortcut add (resid = (x [B*H*W], w [C], b [C])).
    tape (train mode): the layer's backward record is appended to it."""
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
    frozen = not bn.training          # eval mode: only reaches the taped form when the call is differentiable
    if bn.training or tape is not None:
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
        if frozen:                                        # running statistics, not updated
            L.cdm_bn_fwd_frozen(Cout, bn.weight.data_ptr(), bn.bias.data_ptr(), bn.running_mean.data_ptr(),
                                bn.running_var.data_ptr(), float(bn.eps), *[t.data_ptr() for t in st], None, 0, None, s)
        else:
            L.cdm_bn_fwd_finalize(ws.dpart.data_ptr(), nparts, 2, Cout, float(P), bn.weight.data_ptr(),
                                  bn.bias.data_ptr(), _p(bn.running_mean) if track else None,
                                  _p(bn.running_var) if track else None, _p(bn.num_batches_tracked) if track else None,
                                  mom, float(bn.eps), *[t.data_ptr() for t in st], None, 0, None, s)
        scale, shift, flags = st[2], st[3], APPLY_RELU
        if tape is not None:
            wdg = None
            if Cin > 1:
                wdg = E(9 * Cout, Cin)
                L.cdm_pack_conv3x3(Wt.data_ptr(), bt.data_ptr(), Cin, Cout, None, None, None, None, 0.0,
                                   E(9 * Cin, Cout).data_ptr(), None, wdg.data_ptr(), kc, s)
            # (C_in = 1: the NHWC input [B*H*W, 1] is the NCHW map the C_in = 1 weight gradient reads)
            rec = dict(dims=(B, H, W, Cin, Cout), conv=conv, bn=bn, st=st, y=y, pool=pool, wdg=wdg, kc=kc, x=xh,
                       frozen=frozen, resid_w=None if resid is None else resid[1])
            if not tape.ops:
                tape.first_rec = rec
            tape.ops.append(lambda g, rec=rec: _layer_backward(rec, tape, g, tape.need_dx(rec)))
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


def residual_block(blk, xh: torch.Tensor, x_nchw: torch.Tensor, B: int, H: int, W: int, pool: bool = False,
                   tape: "_Tape" = None):
    """ResidualConvBlock.forward (diffusion_utilities.py:39-65) on NHWC xh.  is_res: out = x + x2 (same channels) or
    shortcut(x) + x2, the shortcut a fresh nn.Conv2d(Cin, Cout, 1) drawn from the CPU RNG on every call (:54) — C_in = 1
    inside the conv2 apply (ContextUnet's init_conv), C_in > 1 as a GEMM accumulated onto the output."""
    if not blk.is_res:
        z1 = conv_bn_relu(blk.conv1, xh, B, H, W, tape=tape)
        return conv_bn_relu(blk.conv2, z1, B, H, W, pool=pool, resid=None, tape=tape)
    Cin, Cout = blk.conv1[0].in_channels, blk.conv2[0].out_channels
    if pool:
        raise NotImplementedError("a residual block with the fused MaxPool2d (the reference's UnetDown blocks are not "
                                  "residual)")
    if not blk.same_channels:
        # the reference draws a fresh 1x1 conv on every call (diffusion_utilities.py:54): same CPU RNG consumption
        sc = nn.Conv2d(Cin, Cout, kernel_size=1, stride=1, padding=0)
        sw, sb = sc.weight.detach().reshape(Cout, Cin).to(xh.device), sc.bias.detach().to(xh.device)
        if Cin == 1:
            resid = (x_nchw.reshape(-1).contiguous(), sw.reshape(Cout).contiguous(), sb)
            z1 = conv_bn_relu(blk.conv1, xh, B, H, W, tape=tape)
            return conv_bn_relu(blk.conv2, z1, B, H, W, resid=resid, tape=tape)
        if Cin % 4 or Cout % 4:
            raise NotImplementedError("the HIP residual shortcut GEMM needs channels % 4 == 0")
    L, s = lib(), _s()
    P = B * H * W
    sub = None
    if tape is not None:        # the block's two layers on a tape of their own; the skip joins in one parent op
        sub = _Tape()
        sub.grads = tape.grads
    first = tape is not None and not tape.ops
    z1 = conv_bn_relu(blk.conv1, xh, B, H, W, tape=sub)
    out = conv_bn_relu(blk.conv2, z1, B, H, W, tape=sub)
    if blk.same_channels:       # out += x
        L.cdm_slab_reduce(xh.data_ptr(), 1, P, Cout, out.data_ptr(), Cout, 0, 1, Cout, 1, 1.0, s)
    else:                       # out += x . W^T + b
        swT = torch.empty(Cin, Cout, device=xh.device)
        L.cdm_transpose(sw.contiguous().data_ptr(), Cout, Cin, swT.data_ptr(), s)
        if L.cdm_gemm_f32(xh.data_ptr(), Cin, P, Cin, swT.data_ptr(), Cout, Cout, out.data_ptr(), Cout, sb.data_ptr(),
                          Cout, EPI_ACCUM, 1, None, s):
            raise RuntimeError("cdm_gemm_f32 (residual shortcut) failed")
    if tape is not None:
        def op(g):
            sub.need_input = tape.need_input if first else True
            dx = sub.run(g)
            if dx is None:
                return None
            if blk.same_channels:   # dx += g
                L.cdm_slab_reduce(g.data_ptr(), 1, P, Cout, dx.data_ptr(), Cin, 0, 1, Cout, 1, 1.0, _s())
            elif L.cdm_gemm_f32(g.data_ptr(), Cout, P, Cout, sw.contiguous().data_ptr(), Cin, Cin, dx.data_ptr(), Cin,
                                None, 1, EPI_ACCUM, 1, None, _s()):   # dx += g . W
                raise RuntimeError("cdm_gemm_f32 (residual shortcut backward) failed")
            return dx
        tape.ops.append(op)
    return out


def _new_tape(module: nn.Module, *inputs):
    """A tape when this call must be differentiable (grad enabled, something requires grad), else None.  Eval mode
    records the same tape with BatchNorm frozen on the running statistics."""
    if not torch.is_grad_enabled():
        return None
    if not (any(p.requires_grad for p in module.parameters()) or any(x.requires_grad for x in inputs)):
        return None
    return _Tape()


def residual_block_forward(blk, x: torch.Tensor) -> torch.Tensor:
    x0 = x
    x = _check(x, "ResidualConvBlock")
    B, _, H, W = x.shape
    tape = _new_tape(blk, x0)
    y = residual_block(blk, to_nhwc(x), x, B, H, W, tape=tape)
    Cout = blk.conv2[0].out_channels
    if tape is not None:
        tape.backward = lambda g, need, shapes: [_input_grad(tape, g, need, shapes)]
    return _finish(to_nchw(y, B, H, W, Cout), blk, tape, (x0,))


def unet_down_forward(mod, x: torch.Tensor) -> torch.Tensor:
    """UnetDown.forward (diffusion_utilities.py:114-116): 2 ResidualConvBlocks + MaxPool2d(2)."""
    x0 = x
    x = _check(x, "UnetDown")
    B, _, H, W = x.shape
    if H % 2 or W % 2:
        raise NotImplementedError("the fused MaxPool2d(2) needs even H and W")
    tape = _new_tape(mod, x0)
    z = residual_block(mod.model[0], to_nhwc(x), x, B, H, W, tape=tape)
    z = residual_block(mod.model[1], z, None, B, H, W, pool=True, tape=tape)
    if tape is not None:
        tape.backward = lambda g, need, shapes: [_input_grad(tape, g, need, shapes)]
    return _finish(to_nchw(z, B, H // 2, W // 2, mod.model[1].conv2[0].out_channels), mod, tape, (x0,))


def unet_up_forward(mod, x: torch.Tensor, skip: torch.Tensor) -> torch.Tensor:
    """UnetUp.forward (diffusion_utilities.py:94-100): cat(x, skip) -> ConvTranspose2d(2, 2) -> 2 ResidualConvBlocks."""
    x0, skip0 = x, skip
    x = _check(torch.cat((x.detach(), skip.detach()), 1), "UnetUp")
    L, s = lib(), _s()
    B, Cin, H, W = x.shape
    ct = mod.model[0]
    Cout = ct.out_channels
    if Cin % 4 or Cout % 4:
        raise NotImplementedError("the HIP ConvTranspose path needs channels % 4 == 0")
    tape = _new_tape(mod, x0, skip0)
    wt = torch.empty(Cin, 4 * Cout, device=x.device)
    wtT = torch.empty(4 * Cout, Cin, device=x.device) if tape is not None else None
    L.cdm_pack_convT(ct.weight.detach().contiguous().data_ptr(), Cin, Cout, 4, wt.data_ptr(), _p(wtT), s)
    y = torch.empty(B * 4 * H * W, Cout, device=x.device)
    xh = to_nhwc(x)
    L.cdm_convT2x2_fwd(xh.data_ptr(), B, H, W, Cin, Cin, wt.data_ptr(), ct.bias.detach().data_ptr(), y.data_ptr(),
                       Cout, Cout, None, s)
    if tape is not None:
        tape.ops.append(lambda g: _convT_backward(ct, tape, g, xh, wtT, B, H, W, Cin, Cout))
    z = residual_block(mod.model[1], y, None, B, 2 * H, 2 * W, tape=tape)
    z = residual_block(mod.model[2], z, None, B, 2 * H, 2 * W, tape=tape)
    if tape is not None:
        Cx = x0.shape[1]

        def backward(g, need, shapes):
            dxh = tape.run(to_nhwc(g))                               # NHWC [B*H*W, Cin] of cat(x, skip)
            dcat = to_nchw(dxh, B, H, W, Cin)
            return [dcat[:, :Cx].contiguous() if need[0] else None, dcat[:, Cx:].contiguous() if need[1] else None]
        tape.backward = backward
    return _finish(to_nchw(z, B, 2 * H, 2 * W, mod.model[2].conv2[0].out_channels), mod, tape, (x0, skip0))


def _convT_backward(ct, tape: "_Tape", g, xh, wtT, B, H, W, Cin, Cout):
    """ConvTranspose2d(Cin, Cout, 2, 2) backward (diffusion_utilities.py:86 under autograd): bias and weight gradients,
    and the NHWC gradient of its input."""
    L, s = lib(), _s()
    dev = g.device
    E = lambda *shape: torch.empty(*shape, device=dev)   # noqa: E731
    Ho = 2 * H
    nt = B * _cdiv(Ho * Ho, CHUNK)
    slab = E(nt * Cout)
    L.cdm_reduce_sum(g.data_ptr(), Cout, B, Ho * Ho, Cout, CHUNK, slab.data_ptr(), s)
    ws = _dpart(dev)
    nparts = fold(ws, slab.data_ptr(), nt, 1, Cout, s)
    db = E(Cout)
    L.cdm_slab_sum_all(ws.dpart.data_ptr(), nparts, 1, 0, 1, Cout, db.data_ptr(), 0, 1, 0, s)
    sp = wgrad_splits(B * H * W, Cin, 4 * Cout)
    slw = E(sp * Cin * 4 * Cout)
    L.cdm_convT2x2_wgrad(xh.data_ptr(), B, H, W, Cin, Cin, g.data_ptr(), Cout, Cout, sp, slw.data_ptr(), s)
    dW = E(Cin, Cout, 2, 2)
    L.cdm_slab_reduce(slw.data_ptr(), sp, Cin, 4 * Cout, dW.data_ptr(), 4 * Cout, 1, 4, Cout, 0, 1.0, s)
    dx = E(B * H * W, Cin)
    L.cdm_convT2x2_dgrad(g.data_ptr(), B, H, W, Cout, Cout, wtT.data_ptr(), dx.data_ptr(), Cin, Cin, 0, s)
    tape.add(ct.weight, dW)
    tape.add(ct.bias, db)
    return dx


def _input_grad(tape: "_Tape", g, need, shapes):
    """Replay a single-input block's tape on the NCHW output gradient g; the NCHW input gradient if needed."""
    tape.need_input = need[0]
    dxh = tape.run(to_nhwc(g))
    if not need[0]:
        return None
    B, C, H, W = shapes[0]
    return to_nchw(dxh, B, H, W, C)


def embed_fc_forward(mod, x: torch.Tensor) -> torch.Tensor:
    """EmbedFC.forward (diffusion_utilities.py:137-145): x.view(-1, input_dim) -> Linear -> GELU -> Linear; with
    gradients: cdm_embed_bwd (the engine's EmbedFC backward) on the saved pre-activation and activation, the input
    gradient dpre . W1 by cdm_embed_input_grad (any input_dim)."""
    dev = next(mod.parameters()).device
    x0 = x
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
    grad = torch.is_grad_enabled() and (any(p.requires_grad for p in mod.parameters()) or x0.requires_grad)
    pre = torch.empty(rows, E, device=dev) if grad else None
    hid = torch.empty(rows, E, device=dev) if grad else None
    w1 = l1.weight.detach().contiguous()
    d = Mlp4()
    m = d.m[0]
    m.x, m.rows, m.in_dim, m.E = x.data_ptr(), rows, mod.input_dim, E
    m.w1, m.b1 = w1.data_ptr(), l1.bias.detach().data_ptr()
    m.w2, m.w2t, m.b2 = w2.data_ptr(), w2t.data_ptr(), l2.bias.detach().data_ptr()
    m.pre, m.h = _p(pre), _p(hid)
    m.out = out.data_ptr()
    for k in (1, 2, 3):
        d.m[k].rows = 0
    lib().cdm_embed_fwd(ctypes.addressof(d), _s())  # the descriptor is copied into the launch's kernel arguments
    if not grad:
        return _finish(out, mod)
    tape = _Tape()
    in_dim = mod.input_dim

    def backward(g, need, shapes):
        g = g.reshape(rows, E).contiguous()
        dpre = torch.empty(rows, E, device=dev)
        grads = [torch.empty_like(t) for t in (l1.weight, l1.bias, l2.weight, l2.bias)]
        db = Mlp4()
        mb = db.m[0]
        mb.x, mb.rows, mb.in_dim, mb.E = x.data_ptr(), rows, in_dim, E
        mb.w1, mb.b1, mb.w2, mb.w2t, mb.b2 = w1.data_ptr(), l1.bias.data_ptr(), w2.data_ptr(), w2t.data_ptr(), \
            l2.bias.data_ptr()
        mb.pre, mb.h, mb.dout, mb.dpre = pre.data_ptr(), hid.data_ptr(), g.data_ptr(), dpre.data_ptr()
        mb.dw1, mb.db1, mb.dw2, mb.db2 = [t.data_ptr() for t in grads]
        for k in (1, 2, 3):
            db.m[k].rows = 0
        lib().cdm_embed_bwd(ctypes.addressof(db), _s())
        for p_, g_ in zip((l1.weight, l1.bias, l2.weight, l2.bias), grads):
            tape.add(p_, g_)
        if not need[0]:
            return [None]
        # dx = dpre . W1 for any input_dim (the reference's context embeddings take n_cfeat = 5 or 6): the kernel
        # ContextUnet's dt / dc use, with the second MLP empty
        dx = torch.empty(rows, in_dim, device=dev)
        lib().cdm_embed_input_grad(dpre.data_ptr(), w1.data_ptr(), E, None, None, 0, rows, in_dim, dx.data_ptr(), _s())
        return [dx.reshape(shapes[0])]
    tape.backward = backward
    return _finish(out, mod, tape, (x0,))
