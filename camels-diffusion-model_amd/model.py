"""Drop-in ``ContextUnet`` (ContextUnet.py:5-60) whose forward/backward run on the HIP engine.

Parameter tree, names, shapes, default initialisation order and therefore the seeded weights are
identical to the reference, so ``state_dict()`` / ``load_state_dict()`` are interchangeable with
checkpoints of the reference (156 entries incl. BatchNorm buffers).  The building blocks keep the
reference constructor signatures (diffusion_utilities.py:13-145); inside ContextUnet the network is executed as a
whole by :class:`cdm_amd.engine.UNetEngine`, and a block called on its own runs a forward-only HIP path
(:mod:`cdm_amd.blocks`).

The reference draws a *fresh* random 1x1 shortcut convolution on every forward call
(diffusion_utilities.py:54).  ``shortcut_source`` selects where that draw comes from:
``"cpu"`` (default) consumes the CPU torch RNG exactly as the reference does (bit-compatible
seeding), ``"device"`` draws the same U(-1/sqrt(C), 1/sqrt(C)) distribution (C = in_channels) from on-device
Philox (no host work;
used by the captured train/sample loops).
"""
from __future__ import annotations

import itertools
import math
import os
from typing import Dict, List, Optional

import torch
import torch.nn as nn

from .engine import CONV_MATH, UNetEngine

# ------------------------------------------------------------------------------------------------
# building blocks (constructor-compatible with code/diffusion_utilities.py)
# ------------------------------------------------------------------------------------------------


def _conv_bn_relu(cin: int, cout: int) -> nn.Sequential:
    return nn.Sequential(nn.Conv2d(cin, cout, 3, 1, 1), nn.BatchNorm2d(cout), nn.ReLU())


class _Holder(nn.Module):
    """Inside ContextUnet the engine runs the network as a whole; a block called on its own runs its forward on the
    HIP kernels (cdm_amd.blocks: forward only, fp32 convs, train / eval BatchNorm semantics)."""


class ResidualConvBlock(_Holder):
    """diffusion_utilities.py:13-37 — conv1/conv2 = Conv3x3 -> BatchNorm2d -> ReLU."""

    def __init__(self, in_channels: int, out_channels: int, is_res: bool = False) -> None:
        super().__init__()
        self.same_channels = in_channels == out_channels
        self.is_res = is_res
        self.conv1 = _conv_bn_relu(in_channels, out_channels)
        self.conv2 = _conv_bn_relu(out_channels, out_channels)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        from .blocks import residual_block_forward
        return residual_block_forward(self, x)

    def get_out_channels(self):
        return self.conv2[0].out_channels

    def set_out_channels(self, out_channels):
        """diffusion_utilities.py:72-75: rewrites the conv attributes only (as the reference; weights keep their shape)."""
        self.conv1[0].out_channels = out_channels
        self.conv2[0].in_channels = out_channels
        self.conv2[0].out_channels = out_channels


class UnetUp(_Holder):
    """diffusion_utilities.py:79-100 — ConvTranspose2d(in,out,2,2) + 2 residual-free conv blocks."""

    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.model = nn.Sequential(nn.ConvTranspose2d(in_channels, out_channels, 2, 2),
                                   ResidualConvBlock(out_channels, out_channels),
                                   ResidualConvBlock(out_channels, out_channels))

    def forward(self, x, skip):
        from .blocks import unet_up_forward
        return unet_up_forward(self, x, skip)


class UnetDown(_Holder):
    """diffusion_utilities.py:103-116 — 2 conv blocks + MaxPool2d(2)."""

    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.model = nn.Sequential(ResidualConvBlock(in_channels, out_channels),
                                   ResidualConvBlock(out_channels, out_channels), nn.MaxPool2d(2))

    def forward(self, x):
        from .blocks import unet_down_forward
        return unet_down_forward(self, x)


class EmbedFC(_Holder):
    """diffusion_utilities.py:118-145 — Linear(in,e) -> GELU -> Linear(e,e)."""

    def __init__(self, input_dim, emb_dim):
        super().__init__()
        self.input_dim = input_dim
        self.model = nn.Sequential(nn.Linear(input_dim, emb_dim), nn.GELU(), nn.Linear(emb_dim, emb_dim))

    def forward(self, x):
        from .blocks import embed_fc_forward
        return embed_fc_forward(self, x)


# ------------------------------------------------------------------------------------------------
# engine registry / autograd bridge
# ------------------------------------------------------------------------------------------------
_ENGINES: Dict[tuple, UNetEngine] = {}
_MODEL_UIDS = itertools.count()


def get_engine(n_feat, n_cfeat, height, device, conv_math: str = "fp32", in_channels: int = 1) -> UNetEngine:
    dev = torch.device(device)
    key = (n_feat, n_cfeat, height, dev.type, dev.index if dev.index is not None else torch.cuda.current_device(),
           conv_math, in_channels)
    eng = _ENGINES.get(key)
    if eng is None:
        eng = _ENGINES[key] = UNetEngine(n_feat, n_cfeat, height, dev, conv_math, in_channels)
    return eng


def default_conv_math() -> str:
    """3x3 conv arithmetic used when ContextUnet(conv_math=None): $CDM_CONV_MATH or "h3" (fp32-class scaled
    split-fp16 on the matrix cores; measured more accurate than "x6" and within 4x of torch's CPU fp32 conv
    error, profiles/r1_conv_accuracy.jsonl).  "fp32" selects plain fp32 MFMA."""
    return os.environ.get("CDM_CONV_MATH", "h3")


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


class _UNetFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, holder, x, t, c, sc_w, sc_b, *params):
        mod: "ContextUnet" = holder[0]
        frozen = holder[1]          # eval mode: BatchNorm on the running statistics (batch_norm(training=False))
        eng, P = mod._engine_and_params(image_channels_ok=True)
        s = _stream()
        B = x.shape[0]
        eng.repack(P, True, s)
        ctx.pack_token = eng.train_pack_token = object()   # whose weights the engine's train pack holds
        ws = eng.workspace(B, True, frozen=frozen)
        eps = eng.forward(ws, P, mod._to_engine(x), t, c, sc_w, sc_b, B, s, frozen=frozen)
        ctx.frozen = frozen
        mod._invalidate_eval_pack()
        ctx.state = (mod, eng, ws, P)
        # the engine backward reads the live parameters (BatchNorm weights, ConvT / EmbedFC weights): saved so that
        # autograd's version check raises if one was updated in place between forward and backward
        ctx.save_for_backward(*params)
        return mod._from_engine(eps, B)

    @staticmethod
    def backward(ctx, geps):
        ctx.saved_tensors                   # version check of the parameters
        mod, eng, ws, P = ctx.state
        names = mod._param_names
        if getattr(eng, "train_pack_token", None) is not ctx.pack_token:
            # another forward (another model of this shape, or an eval pack) re-used the engine's packed weights in
            # between: re-pack this model's (unchanged, version-checked) parameters for its dgrads
            eng.repack(P, True, _stream())
            eng.train_pack_token = ctx.pack_token
        G = {n: torch.empty_like(P[n]) for n in names}
        dev = geps.device
        need_x, need_t, need_c = ctx.needs_input_grad[1:4]
        dx = torch.empty(ws.B * mod.h * mod.h * eng.cp, device=dev) if need_x else None
        dt = torch.empty(ws.t_rows, device=dev) if need_t else None
        dc = torch.empty(ws.c_rows, mod.n_cfeat, device=dev) if need_c else None
        ws.frozen = ctx.frozen
        eng.backward(ws, P, mod._to_engine(geps), G, _stream(), dx=None if dx is None else dx.view_as(ws.eps), dt=dt,
                     dc=dc)
        ctx.state = None
        return (None, None if dx is None else mod._from_engine(dx, ws.B), dt, dc, None, None, *[G[n] for n in names])


class ContextUnet(nn.Module):
    """Drop-in for ContextUnet.py:5-60 (same constructor, attributes, state_dict and forward)."""

    def __init__(self, in_channels, n_feat=128, n_cfeat=10, height=64, shortcut_source: str = "cpu",
                 conv_math: Optional[str] = None):
        super().__init__()
        self.conv_math = conv_math or default_conv_math()
        if self.conv_math not in CONV_MATH:
            raise ValueError(f"conv_math must be one of {sorted(CONV_MATH)}")
        self.in_channels, self.n_feat, self.n_cfeat, self.h = in_channels, n_feat, n_cfeat, height
        # construction order == reference order, so seeded default init reproduces its weights
        self.init_conv = ResidualConvBlock(in_channels, n_feat, is_res=True)
        self.down1 = UnetDown(n_feat, n_feat)
        self.down2 = UnetDown(n_feat, 2 * n_feat)
        self.to_vec = nn.Sequential(nn.AvgPool2d(height // 4), nn.GELU())
        self.timeembed1 = EmbedFC(1, 2 * n_feat)
        self.timeembed2 = EmbedFC(1, n_feat)
        self.contextembed1 = EmbedFC(n_cfeat, 2 * n_feat)
        self.contextembed2 = EmbedFC(n_cfeat, n_feat)
        self.up0 = nn.Sequential(nn.ConvTranspose2d(2 * n_feat, 2 * n_feat, height // 4, height // 4),
                                 nn.GroupNorm(8, 2 * n_feat), nn.ReLU())
        self.up1 = UnetUp(4 * n_feat, n_feat)
        self.up2 = UnetUp(2 * n_feat, n_feat)
        self.out = nn.Sequential(nn.Conv2d(2 * n_feat, n_feat, 3, 1, 1), nn.GroupNorm(8, n_feat), nn.ReLU(),
                                 nn.Conv2d(n_feat, in_channels, 3, 1, 1))
        if shortcut_source not in ("cpu", "device"):
            raise ValueError("shortcut_source must be 'cpu' or 'device'")
        self.shortcut_source = shortcut_source
        self._param_names: List[str] = [n for n, _ in self.named_parameters()]
        self._uid = next(_MODEL_UIDS)     # eval-pack cache identity (see _eval_pack_key)
        self._eval_key = None
        self._sc_counter = 0

    # -------------------------------------------------------------------------------------------
    def _engine_and_params(self, image_channels_ok: bool = False):
        """(engine, parameters).  Module calls (forward / backward) take any in_channels; the reference's training loop,
        samplers and likelihood are single-channel (train_diffusion_condition.py:101,301 build in_channels = 1 and draw
        [n, 1, H, W]), and so are this package's graph-captured versions of them."""
        if self.in_channels != 1 and not image_channels_ok:
            raise NotImplementedError("the training loop / samplers / likelihood of the reference (and of this package) "
                                      "are single-channel: ContextUnet(in_channels > 1) runs module calls only")
        P = dict(self.named_parameters())
        P.update(dict(self.named_buffers()))
        dev = P["out.3.weight"].device
        if dev.type != "cuda":
            raise RuntimeError("ContextUnet runs on the MI355X HIP engine: move the module to a cuda device")
        for k, v in P.items():
            if k.endswith("num_batches_tracked"):
                continue
            if v.dtype != torch.float32 or not v.is_contiguous():
                raise RuntimeError(f"{k}: expected contiguous fp32 (got {v.dtype})")
        return get_engine(self.n_feat, self.n_cfeat, self.h, dev, self.conv_math, self.in_channels), P

    def _to_engine(self, x: torch.Tensor) -> torch.Tensor:
        """[B, C, H, W] -> the engine's image layout: [B, H, W] for C = 1 (NCHW == NHWC); NHWC [B*H*W, cp] with zero
        channels up to cp = a multiple of 4 otherwise."""
        B, C, h = x.shape[0], self.in_channels, self.h
        if tuple(x.shape[1:]) != (C, h, h):
            raise ValueError(f"expected x of shape [B, {C}, {h}, {h}], got {tuple(x.shape)}")
        if C == 1:
            return x.reshape(B, h, h).contiguous()
        cp = (C + 3) // 4 * 4
        xe = x.new_zeros(B, h, h, cp)
        xe[..., :C] = x.permute(0, 2, 3, 1)
        return xe.view(B * h * h, cp)

    def _from_engine(self, e: torch.Tensor, B: int) -> torch.Tensor:
        """the engine's image layout -> [B, C, H, W] (inverse of _to_engine)"""
        C, h = self.in_channels, self.h
        if C == 1:
            return e.view(B, 1, h, h)
        return e.view(B, h, h, -1)[..., :C].permute(0, 3, 1, 2).contiguous()

    def _invalidate_eval_pack(self):
        self._eval_key = None

    def _eval_pack_key(self, P):
        # the engine (and its packed eval weights) is shared by every model of one shape: the key names this model, not
        # only its tensors' addresses and versions — a model built after another was freed can receive the same
        # addresses with the same version counters, and would then run on the freed model's stale pack
        return (self._uid,) + tuple((v.data_ptr(), v._version) for v in P.values())

    def draw_shortcut(self, device, n_sets: int = 1):
        """Fresh 1x1 shortcut (diffusion_utilities.py:54).  Returns (w [n_sets*nf*in_channels], b [n_sets*nf])."""
        nf = self.n_feat
        if self.in_channels == nf:
            # diffusion_utilities.py:50-52: same channels -> out = x + x2, no 1x1 conv is built (no RNG draw); the
            # identity weights make the residual apply compute exactly that
            eye = torch.eye(nf, device=device).reshape(-1)
            return eye.repeat(n_sets), torch.zeros(n_sets * nf, device=device)
        if self.shortcut_source == "cpu":
            ws, bs = [], []
            for _ in range(n_sets):
                conv = nn.Conv2d(self.in_channels, nf, kernel_size=1, stride=1, padding=0)
                ws.append(conv.weight.detach().reshape(-1)); bs.append(conv.bias.detach())
            return torch.cat(ws).to(device), torch.cat(bs).to(device)
        from ._lib import lib
        nw = n_sets * nf * self.in_channels
        w = torch.empty(nw + n_sets * nf, device=device)
        self._sc_counter += 1
        # the reference's fresh nn.Conv2d(C, n_feat, 1) draws weight (kaiming_uniform_, a = sqrt(5)) and bias both from
        # U(-1/sqrt(fan_in), 1/sqrt(fan_in)), fan_in = C: U(-1, 1) for the single-channel maps
        bound = 1.0 / math.sqrt(self.in_channels)
        lib().cdm_philox_uniform(w.data_ptr(), w.numel(), -bound, bound, 0x5C0FFEE + id(self) % 65536,
                                 self._sc_counter, None, _stream())
        return w[:nw], w[nw:]

    # -------------------------------------------------------------------------------------------
    def forward(self, x, t, c=None):
        """x [B,in_channels,H,W]; t in [0,1] with B or 1 elements (any shape); c [B|1, n_cfeat] or None (zeros)."""
        eng, P = self._engine_and_params(image_channels_ok=True)
        dev = x.device
        B = x.shape[0]
        x = x.to(torch.float32).contiguous()
        t = torch.as_tensor(t).to(device=dev, dtype=torch.float32).reshape(-1).contiguous()
        if c is not None:
            c = c.to(device=dev, dtype=torch.float32).reshape(-1, self.n_cfeat).contiguous()
        sc_w, sc_b = self.draw_shortcut(dev)
        needs_grad = torch.is_grad_enabled() and (any(p.requires_grad for p in self.parameters())
                                                  or any(v is not None and v.requires_grad for v in (x, t, c)))
        if needs_grad:
            # train mode: batch statistics (and the running-stat update); eval mode under autograd: the same
            # train-structured forward with BatchNorm frozen on the running statistics, differentiable like the
            # reference's eval() module
            return _UNetFunction.apply((self, not self.training), x, t, c, sc_w, sc_b,
                                       *[P[n] for n in self._param_names])
        s = _stream()
        train = self.training
        if train:
            eng.repack(P, True, s)
            self._invalidate_eval_pack()
        else:
            key = self._eval_pack_key(P)
            eng.repack(P, False, s, key=key)
        ws = _cached_ws(eng, B, train)
        if self.in_channels == 1:
            eps = torch.empty(B, 1, self.h, self.h, device=dev)
            eng.forward(ws, P, self._to_engine(x), t, c, sc_w, sc_b, B, s, out=eps.view(B, self.h, self.h))
            return eps
        return self._from_engine(eng.forward(ws, P, self._to_engine(x), t, c, sc_w, sc_b, B, s), B)


_WS: Dict[tuple, object] = {}


def _cached_ws(eng, B, train):
    key = (id(eng), B, train)
    ws = _WS.get(key)
    if ws is None:
        if len(_WS) > 8:
            _WS.clear()
        ws = _WS[key] = eng.workspace(B, train)
    return ws
