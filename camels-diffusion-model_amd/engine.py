"""ContextUnet forward / backward on the HIP kernels (explicit graph, no autograd inside).

Mirrors ContextUnet.forward (ContextUnet.py:42-60, == code/train_diffusion.py:48-66) block by block:

    init_conv (ResidualConvBlock is_res, random 1x1 shortcut)   diffusion_utilities.py:13-65
    down1/down2 (2x RCB + MaxPool2d(2))                          diffusion_utilities.py:103-116
    to_vec (AvgPool2d(h/4) + GELU)                               ContextUnet.py:17
    4x EmbedFC                                                    diffusion_utilities.py:118-145
    up0 (ConvTranspose2d k=h/4 on 1x1, GroupNorm(8), ReLU)       ContextUnet.py:26-30
    FiLM cemb*u + temb, up1/up2 (cat, ConvT 2x2, 2x RCB)         ContextUnet.py:57-58, diffusion_utilities.py:79-100
    out (conv3x3, GroupNorm(8), ReLU, conv3x3 -> 1)              ContextUnet.py:35-40

Memory layout: every activation is NHWC fp32 in HBM.  The three torch.cat calls are eliminated by
giving each concatenation a single buffer whose channel slices are written by their producers:

    catO  [B, H,   H,   2nf] = [ up2 output | init_conv output x0 ]
    catU2 [B, H/2, H/2, 2nf] = [ FiLM2(up1 output) | d1 = down1 output ]
    catU1 [B, H/4, H/4, 4nf] = [ FiLM1(up0 output) | d2 = down2 output ]

Train mode keeps every BatchNorm's pre-norm conv output y (the normalised/ReLU'd activation z is
kept only where the next conv reads it); the backward recomputes relu masks / max-pool argmaxes /
x-hat from y.  Eval mode folds BatchNorm into the conv weights and runs ReLU in the conv epilogue.
"""
from __future__ import annotations

import math
import os
from typing import Dict, Optional

import torch

from ._lib import Mlp4, MlpDesc, lib

BN_EPS = 1e-5
BN_MOM = 0.1
GN_EPS = 1e-5
GN_GROUPS = 8
CHUNK = 128           # pixels per statistics partial (== GEMM M tile)
EPI_RELU, EPI_ACCUM = 1, 2
APPLY_POOL, APPLY_FILM, APPLY_RESID, APPLY_RELU = 1, 2, 4, 8


def _p(t: Optional[torch.Tensor], off: int = 0):
    return None if t is None else t.data_ptr() + 4 * off


class Act:
    """NHWC activation view: channels [off, off+C) of a buffer whose pixel stride is ``ld`` floats."""
    __slots__ = ("buf", "C", "ld", "off")

    def __init__(self, buf: torch.Tensor, C: int, ld: Optional[int] = None, off: int = 0):
        self.buf, self.C, self.ld, self.off = buf, C, (C if ld is None else ld), off

    @property
    def p(self):
        return self.buf.data_ptr() + 4 * self.off

    def sl(self, c0: int, C: int) -> "Act":
        return Act(self.buf, C, self.ld, self.off + c0)


def _cdiv(a, b):
    return (a + b - 1) // b


class LayerSpec:
    """One Conv3x3 -> BatchNorm2d -> ReLU (diffusion_utilities.py:26-37)."""

    def __init__(self, name, cin, cout, S):
        self.name, self.cin, self.cout, self.S = name, cin, cout, S
        self.w, self.b = name + ".0.weight", name + ".0.bias"
        self.bn = name + ".1"
        self.kc = conv_kc(cin, cout)


def conv_kc(cin: int, cout: int) -> int:
    """K order of a conv's packed weights: channel-chunk-major (16) when both channel counts allow."""
    return 16 if (cin % 16 == 0 and cout % 16 == 0) else 0


def conv_layers(nf: int, H: int, cin0: int = 1):
    """The 18 Conv3x3 -> BatchNorm -> ReLU layers in forward order; cin0 = the image channels the init conv reads
    (in_channels, padded to a multiple of 4 when > 1)."""
    L = []

    def rcb(prefix, cin, cout, S):
        L.append(LayerSpec(prefix + ".conv1", cin, cout, S))
        L.append(LayerSpec(prefix + ".conv2", cout, cout, S))

    rcb("init_conv", cin0, nf, H)
    rcb("down1.model.0", nf, nf, H); rcb("down1.model.1", nf, nf, H)
    rcb("down2.model.0", nf, 2 * nf, H // 2); rcb("down2.model.1", 2 * nf, 2 * nf, H // 2)
    rcb("up1.model.1", nf, nf, H // 2); rcb("up1.model.2", nf, nf, H // 2)
    rcb("up2.model.1", nf, nf, H); rcb("up2.model.2", nf, nf, H)
    return L


# 3x3 conv arithmetic: "fp32" = fp32 MFMA (v_mfma_f32_32x32x2_f32); "x6" = fp32-accurate split-bf16
# (6 cross terms on v_mfma_f32_32x32x16_bf16, see csrc/gemm_f32.hip); "h3" = fp32-class scaled fp16
# hi/lo split (3 cross terms on v_mfma_f32_32x32x16_f16; per-tensor power-of-two scale from max|.|);
# "x3" / "bf16" = reduced-precision variants (bf16x3 / plain bf16 operands, fp32 accumulate) for the
# mixed-precision configuration.
CONV_MATH = {"fp32": 0, "x6": 6, "x3": 3, "bf16": 1, "h3": 4}
NT_H3 = 4

MLPS = ("contextembed1", "timeembed1", "contextembed2", "timeembed2")


class UNetEngine:
    """Kernel-level ContextUnet for one (n_feat, n_cfeat, height) on one device."""

    def __init__(self, n_feat: int, n_cfeat: int, height: int, device, conv_math: str = "fp32", in_channels: int = 1):
        # the reference needs height % 4 == 0 (two MaxPool2d(2), AvgPool2d(h/4), ConvTranspose2d(k = h/4):
        # ContextUnet.py:17,27); the LDS-halo / band / fused paths take the map widths they support and every other
        # width runs the generic kernels (round 5: heights 20, 36, 48 tested)
        if n_feat % 8 or height % 4 or height < 4:
            raise ValueError("HIP path needs n_feat % 8 == 0 and height % 4 == 0")
        if conv_math not in CONV_MATH:
            raise ValueError(f"conv_math must be one of {sorted(CONV_MATH)}")
        self.nf, self.ncf, self.H = n_feat, n_cfeat, height
        # image channels (ContextUnet.py:6,14,39).  The reference's call sites all build in_channels = 1, for which the
        # C_in = 1 init-conv kernels and the C_out = 1 out.3 kernels run.  More channels run the general conv kernels
        # on NHWC images padded to cp = a multiple of 4 channels (zero image channels, zero weight columns / rows)
        if in_channels < 1:
            raise ValueError("in_channels must be >= 1")
        self.cimg = in_channels
        self.cp = 1 if in_channels == 1 else _cdiv(in_channels, 4) * 4
        self.conv_math = conv_math
        self.nterm = CONV_MATH[conv_math]
        # the 16-bit-MFMA kernel family with every train-mode fusion: h3 (fp32-class) and bf16 (C4 mixed precision)
        self.x16 = self.nterm in (1, NT_H3)
        self.h3 = self.nterm == NT_H3
        # BatchNorm backward fused into the staging of the layer's dgrad / wgrad (dy never written);
        # $CDM_FUSE_BN_BWD=0 keeps the separate apply kernel (A/B checks)
        self.fuse_bn_bwd = self.x16 and os.environ.get("CDM_FUSE_BN_BWD", "1") != "0"
        # a dense BatchNorm + ReLU applied inside the next conv's staging ($CDM_FUSE_BN_FWD=0: apply kernel)
        self.fuse_bn_fwd = self.x16 and os.environ.get("CDM_FUSE_BN_FWD", "1") != "0"
        # a fused layer's dgrad also stores the dy its staging computes (the BN backward of g), and the weight gradient
        # stages that dy instead of evaluating the BN backward again in each of its 3 kernel-row blocks
        # ($CDM_DY_STORE=0 / 1; same-box A/B, 2 runs each: C4 29.64-29.89 -> 29.02-29.04 ms per step, C2 50.57-50.62 ->
        # 50.36-50.37 ms, profiles/r4_ab_dy_store_ks4.txt)
        self.dy_store = self.x16 and os.environ.get("CDM_DY_STORE", "1") == "1"
        # a fused producer's BN-backward channel sums accumulated in its consumer's weight-gradient X staging (which
        # stages the producer's y anyway), after the consumer's dgrad wrote the producer's g: no separate pass over g and
        # y.  Round 3 kept it off for h3 (C2 52.56 -> 55.07 ms: the h3 weight gradient with the BN-backward dy staging sat
        # at the 256-VGPR limit); since round 4 the weight gradient stages the dy the dgrad stored (dy_store) and the
        # sums fit (250 VGPRs, no spill): same-box A/B, 2 runs each, C2 50.36-50.38 -> 49.39-49.45 ms per step
        # (profiles/r4_ab_sums_dy_pass.txt).  $CDM_FUSE_BN_SUMS=0 / 1 forces it.
        env = os.environ.get("CDM_FUSE_BN_SUMS")
        self.fuse_bn_sums = self.x16 and (env == "1" if env is not None else (self.dy_store or not self.h3))
        # init_conv.conv1's BN backward inside its weight-gradient kernel ($CDM_FUSE_CIN1_BWD=0: the apply kernel)
        self.fuse_cin1_bwd = os.environ.get("CDM_FUSE_CIN1_BWD", "1") != "0"
        # C4 mixed precision (bf16 arithmetic, train mode): the fused Conv -> BN -> ReLU chain's pre-norm outputs y and
        # their gradients g are stored as bf16 (torch.autocast keeps conv outputs and their gradients in bf16), halving
        # the bytes every fused conv stages; BN statistics, accumulators, master weights stay fp32.  The chain's ends
        # (concatenation slices, pool / FiLM / residual outputs, the C_in = 1 init conv) stay fp32.
        # $CDM_ACT16=0 keeps fp32 activations (A/B checks).
        self.act16 = self.nterm == 1 and os.environ.get("CDM_ACT16", "1") != "0"
        # bf16 (one-term) arithmetic: dy of a fused layer by a separate elementwise pass (cdm_bn_bwd_dy) and the
        # dgrad on the forward's staging schedule (halo two chunks ahead) instead of the BN-backward staging.  Round 4
        # kept it off (C4 28.20 -> 28.31-28.33 ms: the pass took 213 us per 64^2 layer, profiles/r4_ab_sums_dy_pass.txt);
        # round 5 loads the pass's per-channel coefficients once per thread instead of per element, and it pays: same-box
        # A/B, 2 runs each, C4 27.33-27.38 -> 26.86-26.89 ms per step (profiles/r5_ab_dy_pass.txt).  $CDM_DY_PASS=0: off
        self.dy_pass = self.dy_store and self.nterm == 1 and os.environ.get("CDM_DY_PASS", "1") == "1"
        # train: out.1's GroupNorm + ReLU inside out.3's forward and weight-gradient staging, zO never written
        # ($CDM_FUSE_GN_OUT=0: the apply kernel writes zO)
        self.fuse_gn_out = os.environ.get("CDM_FUSE_GN_OUT", "1") != "0"
        # eval: the pool / FiLM / residual applies in the conv epilogue (fuses_eval)
        self.fuse_eval = self.x16 and os.environ.get("CDM_FUSE_EVAL", "1") != "0"
        self.device = torch.device(device)
        self.layers = conv_layers(n_feat, height, self.cp)
        self.L = {l.name: l for l in self.layers}
        self.KK0 = (height // 4) ** 2
        # up0 on large maps (config 5: k = 64, 1.07 G weights): VALU kernels over the weights in their reference layout
        # (cdm_up0_fwd / cdm_up0_wgrad) and one W^T for the input gradient, instead of two 4.3 GB repacks per step
        self.up0_large = self.KK0 >= 1024 and self.KK0 % 256 == 0 and (2 * n_feat) % 16 == 0 and 2 * n_feat <= 512
        self.kc_out0 = conv_kc(2 * n_feat, n_feat)
        self.pk: Dict[str, torch.Tensor] = {}
        self._pk_key = None
        self.train_pack_token = None     # identity of the autograd forward whose train pack pk holds (model.py)
        self._ones =torch.ones(4 * n_feat, device=self.device)
        self._zeros = torch.zeros(4 * n_feat, device=self.device)
        self._amax = torch.zeros(2, device=self.device)     # h3: max|A|, max|B| of the current launch
        # h3 train: batched repack (3 launches per step); $CDM_BATCH_REPACK=0 keeps the per-layer launches (A/B)
        self.batch_repack = os.environ.get("CDM_BATCH_REPACK", "1") != "0"
        # measurement hook: probe(args) before every 3x3 conv launch, args = the _conv3x3 arguments (bench.py replays
        # the dominant conv's launches of a real train step on their real operands); None in production
        self.launch_probe = None
        # diagnostic hook: stage_probe(stage, ws) at fixed points of the forward ("x0", "d1", "d2", "emb", "film2", "u3";
        # tools/t1500_steps.py substitutes reference values there to locate an error source); None in production
        self.stage_probe = None
        self._batch_key = None

    # ------------------------------------------------------------------------------------------
    # weight packing (OIHW / [Cin][Cout][kh][kw] -> GEMM layouts; eval: BatchNorm folded)
    # ------------------------------------------------------------------------------------------
    def _repack_h3_train_batched(self, P, stream: int):
        """h3 / bf16 train mode: every 3x3 conv with C_in > 1 (and out.0) repacked in 3 launches — clear the max|W|
        slots, max|W| per layer, the split images straight from OIHW (cdm_pack_split_conv3x3_batch; bf16: the one-term
        hi plane, round 5 — it replaced 40 split + 18 pack launches per C4 step)."""
        nf = self.nf
        specs = [(l.name, self._layer_w(P, l), l.cin, l.cout, l.kc) for l in self.layers if l.cin > 1]
        specs.append(("out.0", P["out.0.weight"], 2 * nf, nf, self.kc_out0))
        key = tuple(w.data_ptr() for _, w, *_ in specs)
        if self._batch_key != key:
            import ctypes

            class Job(ctypes.Structure):
                _fields_ = [("W", ctypes.c_void_p), ("Cin", ctypes.c_int), ("Cout", ctypes.c_int), ("kc", ctypes.c_int),
                            ("pad", ctypes.c_int), ("wpk_x", ctypes.c_void_p), ("wdg_x", ctypes.c_void_p),
                            ("amax", ctypes.c_void_p)]
            assert ctypes.sizeof(Job) == 48
            slots = torch.zeros(len(specs), device=self.device)
            arr = (Job * len(specs))()
            for i, (name, W, cin, cout, kc) in enumerate(specs):
                wx = self._buf(name + ".wpk_x", (_cdiv(9 * cin, 16) * 3 * cout * 16,), torch.bfloat16)
                wdx = self._buf(name + ".wdg_x", (_cdiv(9 * cout, 16) * 3 * cin * 16,), torch.bfloat16)
                self.pk[name + ".wpk_x"], self.pk[name + ".wdg_x"] = wx, wdx
                self.pk[name + ".wpk_amax"] = self.pk[name + ".wdg_amax"] = slots[i:i + 1]
                arr[i] = Job(W.data_ptr(), cin, cout, kc, 0 if self.h3 else 1, wx.data_ptr(), wdx.data_ptr(),
                             slots.data_ptr() + 4 * i)
            raw = bytes(memoryview(arr).cast("B"))
            self._batch_jobs = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(self.device)
            self._batch_slots, self._batch_n = slots, len(specs)
            self._batch_max = max(cin * cout * 9 for _, _, cin, cout, _ in specs)
            self._batch_key = key
        lb = lib()
        lb.cdm_zero_f32(_p(self._batch_slots), self._batch_n, stream)
        lb.cdm_pack_split_conv3x3_batch(_p(self._batch_jobs), self._batch_n, self._batch_max, stream)

    def repack(self, P: Dict[str, torch.Tensor], train: bool, stream: int, key=None):
        if key is not None and self._pk_key == (key, train):
            return
        self.train_pack_token = None          # the pack changes owner (model.py re-packs before a stale backward)
        lb = lib(); nf = self.nf
        batched = train and self.x16 and self.batch_repack
        if batched:
            self._repack_h3_train_batched(P, stream)
        for l in self.layers:
            if batched and l.cin > 1:
                continue
            W, b = self._layer_w(P, l), P[l.b]
            if train:
                wpk = self._buf(l.name + ".wpk", (9 * l.cin, l.cout))
                wdg = (self._buf(l.name + ".wdg", (9 * l.cout, l.cin))) if l.cin > 1 else None
                lb.cdm_pack_conv3x3(_p(W), _p(b), l.cin, l.cout, None, None, None, None, 0.0, _p(wpk), None,
                                    _p(wdg), l.kc, stream)
                self.pk[l.name + ".wpk"] = wpk
                if wdg is not None:
                    self.pk[l.name + ".wdg"] = wdg
                    self._split(l.name + ".wpk", 9 * l.cin, l.cout, stream)
                    self._split(l.name + ".wdg", 9 * l.cout, l.cin, stream)
            else:
                wpk = self._buf(l.name + ".wpk_e", (9 * l.cin, l.cout))
                bpk = self._buf(l.name + ".bpk_e", (l.cout))
                bn = l.bn
                lb.cdm_pack_conv3x3(_p(W), _p(b), l.cin, l.cout, _p(P[bn + ".weight"]), _p(P[bn + ".bias"]),
                                    _p(P[bn + ".running_mean"]), _p(P[bn + ".running_var"]), BN_EPS, _p(wpk),
                                    _p(bpk), None, l.kc, stream)
                self.pk[l.name + ".wpk_e"] = wpk
                self.pk[l.name + ".bpk_e"] = bpk
                if l.cin > 1:
                    self._split(l.name + ".wpk_e", 9 * l.cin, l.cout, stream)
        # out.0 (GroupNorm follows: never folded)
        if not batched:
            wpk = self._buf("out.0.wpk", (9 * 2 * nf, nf))
            wdg = self._buf("out.0.wdg", (9 * nf, 2 * nf))
            lb.cdm_pack_conv3x3(_p(P["out.0.weight"]), _p(P["out.0.bias"]), 2 * nf, nf, None, None, None, None, 0.0,
                                _p(wpk), None, _p(wdg) if train else None, self.kc_out0, stream)
            self.pk["out.0.wpk"], self.pk["out.0.wdg"] = wpk, wdg
            self._split("out.0.wpk", 9 * 2 * nf, nf, stream)
            if train:
                self._split("out.0.wdg", 9 * nf, 2 * nf, stream)
        if self.cp > 1:
            # out.3 (n_feat -> in_channels) on the general conv kernels: weights / bias padded to cp output channels
            cp, C = self.cp, self.cimg
            w3 = self._buf("out.3.wpad", (cp, nf, 3, 3))
            b3 = self._buf("out.3.bpad", (cp,))
            w3[C:].zero_(); w3[:C].copy_(P["out.3.weight"])
            b3[C:].zero_(); b3[:C].copy_(P["out.3.bias"])
            self.pk["out.3.wpad"], self.pk["out.3.bpad"] = w3, b3
            wpk = self._buf("out.3.wpk", (9 * nf, cp))
            wdg = self._buf("out.3.wdg", (9 * cp, nf))
            lb.cdm_pack_conv3x3(_p(w3), _p(b3), nf, cp, None, None, None, None, 0.0, _p(wpk), None,
                                _p(wdg) if train else None, conv_kc(nf, cp), stream)
            self.pk["out.3.wpk"], self.pk["out.3.wdg"] = wpk, wdg
            self._split("out.3.wpk", 9 * nf, cp, stream)
            if train:
                self._split("out.3.wdg", 9 * cp, nf, stream)
        for name, cin in (("up1.model.0", 4 * nf), ("up2.model.0", 2 * nf)):
            wt = self._buf(name + ".wt", (cin, 4 * nf))
            wtT = self._buf(name + ".wtT", (4 * nf, cin))
            lb.cdm_pack_convT(_p(P[name + ".weight"]), cin, nf, 4, _p(wt), _p(wtT) if train else None, stream)
            self.pk[name + ".wt"], self.pk[name + ".wtT"] = wt, wtT
            if self.x16:
                self._split(name + ".wt", cin, 4 * nf, stream)
                if train:
                    self._split(name + ".wtT", 4 * nf, cin, stream)
        c0 = 2 * nf
        if self.up0_large:
            pass   # W[ci][(co, ij)] is used in place (B > 16 input gradients build their W^T in the backward)
        else:
            w0 = self._buf("up0.wt", (c0, self.KK0 * c0))
            w0T = self._buf("up0.wtT", (self.KK0 * c0, c0))
            lb.cdm_pack_convT(_p(P["up0.0.weight"]), c0, c0, self.KK0, _p(w0), _p(w0T) if train else None, stream)
            self.pk["up0.wt"], self.pk["up0.wtT"] = w0, w0T
            if self.x16:    # the forward GEMM on the 16-bit matrix cores (cdm_gemm_x16)
                self._split("up0.wt", c0, self.KK0 * c0, stream)
        for m in MLPS:
            w2 = P[m + ".model.2.weight"]
            E = w2.shape[0]
            w2t = self._buf(m + ".w2t", (E, E))
            lb.cdm_transpose(_p(w2), E, E, _p(w2t), stream)
            self.pk[m + ".w2t"] = w2t
        self._pk_key = (key, train) if key is not None else None

    def _layer_w(self, P, l: "LayerSpec") -> torch.Tensor:
        """Conv l's OIHW weights; the init conv's with zero columns for the padded image channels (in_channels > 1)."""
        W = P[l.w]
        if l is not self.layers[0] or self.cp == self.cimg:
            return W
        wp = self.pk["init.wpad"] = self._buf("init.wpad", (self.nf, self.cp, 3, 3))
        wp[:, self.cimg:].zero_()
        wp[:, :self.cimg].copy_(W)
        return wp

    def invalidate(self):
        """Parameters changed behind torch's version counters (fused Adam): drop the cached eval pack."""
        self._pk_key = None

    def _buf(self, name, shape, dtype=torch.float32):
        shape = (shape,) if isinstance(shape, int) else tuple(shape)
        t = self.pk.get(name)
        if t is None or tuple(t.shape) != tuple(shape) or t.dtype != dtype:
            t = torch.empty(*shape, device=self.device, dtype=dtype)
        return t

    def _split(self, name, K, N, stream):
        """16-bit split of the packed fp32 [K][N] weights pk[name] -> pk[name + "_x"] (bf16 hi/mid/lo, or
        for h3 the scaled fp16 hi/lo with max|W| in pk[name + "_amax"])."""
        if not self.nterm:
            return
        xb = self._buf(name + "_x", (_cdiv(K, 16) * 3 * N * 16,), torch.bfloat16)
        if self.nterm == NT_H3:
            am = self._buf(name + "_amax", (1,))
            lib().cdm_amax_f32(_p(self.pk[name]), K, N, N, _p(am), 0, stream)
            lib().cdm_split_f16x2(_p(self.pk[name]), N, K, N, _p(am), _p(xb), stream)
            self.pk[name + "_amax"] = am
        else:
            lib().cdm_split_bf16x3(_p(self.pk[name]), N, K, N, _p(xb), stream)
        self.pk[name + "_x"] = xb

    def _wamax(self, key):
        """Device max|W| of the split weights pk[key + "_x"] (h3 scale), None for the other arithmetics."""
        return _p(self.pk[key + "_amax"]) if self.h3 else None

    def conv3x3(self, key, x_p, B, S, cin, ldx, bias_p, y_p, ldy, cout, flags, stats_p, stats_ld, kc, s,
                amax_x=None, amax_y=None, pre=None, ymm=None, dt=0):
        """3x3 conv (fwd or dgrad) with the packed weights pk[key], in this engine's conv arithmetic.

        h3 only: amax_x = device max|x| written by x's producer (None: measured here by a separate pass);
        amax_y = slot that receives max|y| for the next conv; pre = (scale, shift) pointers: the input is
        relu(x * scale + shift) of the previous layer's pre-norm output, applied while staging; ymm = (ptr, ld):
        per-channel max / min keys of y for the next layer's fused apply."""
        args = (key, x_p, B, S, cin, ldx, bias_p, y_p, ldy, cout, flags, stats_p, stats_ld, kc, s, amax_x, amax_y,
                pre, ymm, dt)
        if self.launch_probe is not None:
            self.launch_probe(args)
        self._conv3x3(*args)

    def _conv3x3(self, key, x_p, B, S, cin, ldx, bias_p, y_p, ldy, cout, flags, stats_p, stats_ld, kc, s, amax_x,
                 amax_y, pre, ymm, dt=0):
        """dt (bf16 activations, C4): bit 0 the source holds bf16, bit 1 the output is stored as bf16."""
        if self.x16:
            if self.h3 and amax_x is None:
                assert pre is None
                amax_x = _p(self._amax)
                lib().cdm_amax_f32(x_p, B * S * S, cin, ldx, amax_x, 0, s)
            if pre is not None or ymm is not None:
                ps, pt = pre if pre is not None else (None, None)
                ym, yld = ymm if ymm is not None else (None, 0)
                lib().cdm_conv3x3_fwd_x16_ex(x_p, B, S, S, cin, ldx, ps, pt, _p(self.pk[key + "_x"]), amax_x,
                                             self._wamax(key), bias_p, y_p, ldy, cout, flags, stats_p, stats_ld, kc,
                                             amax_y, ym, yld, self.nterm, dt, s)
                return
            lib().cdm_conv3x3_fwd_x16(x_p, B, S, S, cin, ldx, _p(self.pk[key + "_x"]), amax_x, self._wamax(key),
                                      bias_p, y_p, ldy, cout, flags, stats_p, stats_ld, kc, amax_y, self.nterm, dt, s)
        elif self.nterm:
            lib().cdm_conv3x3_fwd_x3(x_p, B, S, S, cin, ldx, _p(self.pk[key + "_x"]), bias_p, y_p, ldy, cout, flags,
                                     stats_p, stats_ld, kc, self.nterm, s)
        else:
            lib().cdm_conv3x3_fwd(x_p, B, S, S, cin, ldx, _p(self.pk[key]), bias_p, y_p, ldy, cout, flags, stats_p,
                                  stats_ld, kc, s)

    def halo_addressable(self, B: int, S: int) -> bool:
        """The LDS-halo conv addresses its sources by 32-bit byte offsets: B*S*S pixels x the widest row of any
        activation / gradient buffer at that resolution (2 n_feat floats; 4 n_feat at H/4, catU1) must stay below
        4 GiB for the fused (halo-only) paths."""
        ld = (4 if S == self.H // 4 else 2) * self.nf
        return B * S * S * ld * 4 < 2 ** 32

    def fuses_bn_fwd(self, l: "LayerSpec", kind: str, B: int = 1) -> bool:
        """Producer l's train-mode BatchNorm apply (z = relu(y s + t)) runs inside the staging of the next conv (its
        forward and its weight gradient): z is never written.  Needs the LDS-halo path for both convs (max / min
        epilogue on l, BN-ReLU staging on the consumer) and the kernel-row weight gradient for the consumer."""
        if not (self.fuse_bn_fwd and kind == "dense" and self.halo_addressable(B, l.S)):
            return False
        if l.cin == 1 and os.environ.get("CDM_FUSE_CIN1_FWD", "1") == "0":   # A/B switch of the init conv's fusion
            return False
        i = self.layers.index(l)
        if i + 1 >= len(self.layers):
            return False
        c = self.layers[i + 1]
        widths = (32, 64, 128, 256) if self.h3 else (32, 64)     # the wide-row LDS-halo conv is h3-only
        halo = lambda L: L.kc == 16 and L.S in widths and (L.S * L.S) % 256 == 0   # noqa: E731
        # the producer's max / min of y: from its conv epilogue (LDS-halo path), or from the statistics pass of the
        # C_in = 1 init conv (cdm_reduce_stats_mm)
        return ((l.cin == 1 or halo(l)) and halo(c) and c.cin == l.cout and c.cin <= 256 and c.cin % 128 == 0
                and c.cout % 128 == 0 and c.S == l.S)

    def fuses_gn_out(self, train: bool) -> bool:
        """out.1's GroupNorm + ReLU runs inside out.3's kernels (forward; train: and its weight gradient): zO is never
        written, and its workspace buffer is not allocated."""
        nf, H = self.nf, self.H
        return (self.cp == 1 and (not train or self.fuse_gn_out) and nf % 16 == 0 and H <= 256 and 256 % H == 0)

    def fuses_bn_bwd(self, l: "LayerSpec", kind: str, B: int = 1) -> bool:
        """Layer l's BN backward runs inside its dgrad / wgrad staging (cdm_conv3x3_*_h3_bnbwd)."""
        return (self.fuse_bn_bwd and kind in ("dense", "plain", "resid") and l.cin > 1 and l is not self.layers[0]
                and l.S in ((32, 64, 128) if self.h3 else (32, 64))
                and self.halo_addressable(B, l.S)
                and l.kc == 16 and l.cin % 128 == 0 and l.cout % 128 == 0 and l.cout <= 256)

    # h3 operand maxima: one device slot per producer, zeroed at the start of every forward --------------
    def _slot(self, ws, key):
        """Pointer to the amax slot `key` of this workspace (None unless the arithmetic is h3)."""
        if self.nterm != NT_H3:
            return None
        i = ws.aslot.get(key)
        if i is None:
            i = ws.aslot[key] = len(ws.aslot)
            assert i < ws.amax.numel()
        return _p(ws.amax) + 4 * i

    # producers writing slices of one concatenation buffer share that buffer's slot (its consumers read the
    # whole buffer, or a slice whose max the shared slot bounds from above — harmless for the scale)
    _CAT_SLOT = {"init_conv.conv2": "catO", "up2.model.2.conv2": "catO", "down1.model.1.conv2": "catU2",
                 "up1.model.2.conv2": "catU2", "down2.model.1.conv2": "catU1"}

    def _dst_slot(self, ws, l: "LayerSpec"):
        return self._slot(ws, self._CAT_SLOT.get(l.name, "z:" + l.name))

    def _src_slot(self, ws, l: "LayerSpec"):
        special = {"down1.model.0.conv1": "catO", "down2.model.0.conv1": "catU2",
                   "up1.model.1.conv1": "yT1", "up2.model.1.conv1": "yT2"}
        if l.name in special:
            return self._slot(ws, special[l.name])
        i = self.layers.index(l)
        if i == 0:
            return None            # the image (in_channels > 1): its max is measured by the conv call
        prev = self.layers[i - 1]
        return self._dst_slot(ws, prev)

    # ------------------------------------------------------------------------------------------
    def workspace(self, B: int, train: bool, frozen: bool = False) -> "Workspace":
        """frozen: a train-structured workspace for the forward / backward of model.eval() under autograd (BatchNorm on
        the running statistics); it keeps fp32 activations under C4's bf16 arithmetic, like the no-grad eval path, so an
        eval model returns the same eps whether or not autograd records it."""
        return Workspace(self, B, train, frozen)

    # ------------------------------------------------------------------------------------------
    # forward
    # ------------------------------------------------------------------------------------------
    def forward(self, ws: "Workspace", P, x: torch.Tensor, t_in: torch.Tensor, c_in: Optional[torch.Tensor],
                sc_w: torch.Tensor, sc_b: torch.Tensor, sc_split: int, stream: int, out: Optional[torch.Tensor] = None,
                frozen: bool = False):
        """x [B,H,W] fp32 (C=1, NCHW == NHWC; in_channels > 1: NHWC [B*H*W, cp] with zero padding channels), t_in [rows_t]
        (rows 1 or B), c_in [rows_c, ncf] or None (zeros).

        sc_w/sc_b: shortcut 1x1 conv weights, [2, nf] when sc_split < B (CFG halves) else [nf]-shaped.
        frozen (train-mode workspace only): BatchNorm with the running statistics, not updated — the forward of
        model.eval() kept for a backward (backward(..., frozen=True)).
        Returns eps [B, H, W] (in_channels > 1: NHWC [B*H*W, cp]; written into ``out`` when given)."""
        lb = lib(); s = stream
        nf, H, B = self.nf, self.H, ws.B
        H1, H2 = H // 2, H // 4
        train = ws.train
        assert train or not frozen
        assert not (frozen and ws.act16), "eval-mode forwards keep fp32 activations: use workspace(B, True, frozen=True)"
        ws.frozen = frozen
        eps = out if out is not None else ws.eps
        ws.x_in = x
        if self.cp > 1:
            assert x.numel() == B * H * H * self.cp
            ws.src["init_conv.conv1"] = Act(x, self.cp)
        ws.sc_pending = (sc_w, sc_b, sc_split)
        if self.nterm == NT_H3:
            lb.cdm_zero_f32(_p(ws.amax), ws.amax.numel(), s)
        if train and ws.fused_fwd and self.h3:
            half = ws.ymm.numel() // 2
            lb.cdm_fill_i32(_p(ws.ymm), half, -2 ** 31, s)               # max keys
            lb.cdm_fill_i32(_p(ws.ymm) + 4 * half, half, 2 ** 31 - 1, s)  # min keys
        # ---------------- encoder ----------------
        probe = self.stage_probe or (lambda stage, ws_: None)
        for i, l in enumerate(self.layers[:10]):
            self._conv_bn_fwd(ws, P, l, s, x)
            if i in (1, 5, 9):
                probe({1: "x0", 5: "d1", 9: "d2"}[i], ws)
        # ---------------- to_vec ----------------
        d2 = ws.catU1.sl(2 * nf, 2 * nf)
        lb.cdm_reduce_sum(d2.p, d2.ld, B, H2 * H2, 2 * nf, H2 * H2, _p(ws.hsum), s)
        lb.cdm_avgpool_gelu_fin(_p(ws.hsum), B, 2 * nf, H2 * H2, _p(ws.hpre), _p(ws.hv), s)
        # ---------------- embeddings ----------------
        rows_t = t_in.numel()
        if c_in is None:
            c_in = ws.c_zero
        rows_c = c_in.shape[0]
        ws.t_rows, ws.c_rows = rows_t, rows_c
        ws.t_x, ws.c_x = t_in, c_in
        d = Mlp4()
        for k, m in enumerate(MLPS):
            is_t = m.startswith("time")
            E = (2 if m.endswith("1") else 1) * nf
            md = d.m[k]
            md.x = _p(t_in if is_t else c_in); md.rows = rows_t if is_t else rows_c
            md.in_dim = 1 if is_t else self.ncf; md.E = E
            md.w1 = _p(P[m + ".model.0.weight"]); md.b1 = _p(P[m + ".model.0.bias"])
            md.w2 = _p(P[m + ".model.2.weight"]); md.w2t = _p(self.pk[m + ".w2t"]); md.b2 = _p(P[m + ".model.2.bias"])
            md.pre = _p(ws.emb_pre[m]) if train else None
            md.h = _p(ws.emb_h[m]) if train else None
            md.out = _p(ws.emb[m])
        lb.cdm_embed_fwd(ctypes_addr(d), s)
        ws._mlp = d
        probe("emb", ws)
        # ---------------- up0: ConvT(k=h/4) on the 1x1 map, GroupNorm(8), ReLU, FiLM1 -> catU1[:, :2nf] ----
        c0 = 2 * nf
        if self.up0_large:
            lb.cdm_up0_fwd(_p(ws.hv), B, c0, _p(P["up0.0.weight"]), self.KK0, _p(P["up0.0.bias"]), _p(ws.y0), s)
        elif self.x16:
            # round 5: h3 / bf16 on the matrix cores (the fp32 MFMA GEMM took 105 us per sampling step at B = 256)
            am_hv = None
            if self.h3:
                am_hv = _p(self._amax)
                lb.cdm_amax_f32(_p(ws.hv), B, c0, c0, am_hv, 0, s)
            lb.cdm_gemm_x16(_p(ws.hv), c0, B, c0, _p(self.pk["up0.wt_x"]), am_hv, self._wamax("up0.wt"),
                            self.KK0 * c0, _p(ws.y0), self.KK0 * c0, _p(P["up0.0.bias"]), c0, None, self.nterm, s)
        else:
            lb.cdm_gemm_f32(_p(ws.hv), c0, B, c0, _p(self.pk["up0.wt"]), self.KK0 * c0, self.KK0 * c0, _p(ws.y0),
                            self.KK0 * c0, _p(P["up0.0.bias"]), c0, 0, 1, None, s)
        self._gn_fwd(ws, P, "up0.1", Act(ws.y0, c0), B, H2, c0, ws.gn0, stats_from_conv=False, stream=s)
        ce1, te1 = ws.emb["contextembed1"], ws.emb["timeembed1"]
        u1 = ws.catU1.sl(0, c0)
        lb.cdm_norm_apply_fwd(APPLY_FILM | APPLY_RELU, _p(ws.y0), c0, B, H2, H2, c0, _p(ws.gn0["scale"]),
                              _p(ws.gn0["shift"]), c0, _p(ce1), c0 if rows_c > 1 else 0, _p(te1),
                              c0 if rows_t > 1 else 0, None, None, None, 0, u1.p, u1.ld, self._slot(ws, "catU1"), s)
        # ---------------- up1 ----------------
        self.convT2x2(ws, "up1.model.0", ws.catU1, B, H2, 4 * nf, P, ws.yT1, "catU1", "yT1", s)
        for l in self.layers[10:14]:
            self._conv_bn_fwd(ws, P, l, s, x)
        probe("film2", ws)
        # ---------------- up2 ----------------
        self.convT2x2(ws, "up2.model.0", ws.catU2, B, H1, 2 * nf, P, ws.yT2, "catU2", "yT2", s)
        for l in self.layers[14:18]:
            self._conv_bn_fwd(ws, P, l, s, x)
        probe("u3", ws)
        # ---------------- out ----------------
        self.conv3x3("out.0.wpk", ws.catO.p, B, H, 2 * nf, 2 * nf, _p(P["out.0.bias"]), _p(ws.yO), nf, nf, 0,
                     _p(ws.slab), nf, self.kc_out0, s, amax_x=self._slot(ws, "catO"))
        probe("yO", ws)
        # out.1's GroupNorm statistics come from out.0's epilogue partials (128-pixel tiles) when no tile spans two images
        self._gn_fwd(ws, P, "out.1", Act(ws.yO, nf), B, H, nf, ws.gnO, stats_from_conv=(H * H) % CHUNK == 0, stream=s)
        if self.fuses_gn_out(train):
            # out.1's GroupNorm + ReLU applied in out.3's staging (train: and in out.3's weight gradient): zO never
            # written
            lb.cdm_conv3x3_cout1_fwd_gn(_p(ws.yO), nf, B, H, H, nf, _p(ws.gnO["scale"]), _p(ws.gnO["shift"]),
                                        _p(P["out.3.weight"]), _p(P["out.3.bias"]), _p(eps), s)
            ws.zO_fused = train
            return eps
        ws.zO_fused = False
        zslot = self._slot(ws, "zO") if self.cp > 1 else None
        lb.cdm_norm_apply_fwd(APPLY_RELU, _p(ws.yO), nf, B, H, H, nf, _p(ws.gnO["scale"]), _p(ws.gnO["shift"]), nf,
                              None, 0, None, 0, None, None, None, 0, _p(ws.zO), nf, zslot, s)
        if self.cp > 1:   # out.3: n_feat -> in_channels (padded to cp) on the general conv kernels
            self.conv3x3("out.3.wpk", _p(ws.zO), B, H, nf, nf, _p(self.pk["out.3.bpad"]), _p(eps), self.cp, self.cp, 0,
                         None, 0, conv_kc(nf, self.cp), s, amax_x=zslot)
            return eps
        lb.cdm_conv3x3_cout1_fwd(_p(ws.zO), nf, B, H, H, nf, _p(P["out.3.weight"]), _p(P["out.3.bias"]), _p(eps), s)
        return eps

    def convT2x2(self, ws, name, x: Act, B, Hin, cin, P, y, src_slot, dst_slot, s):
        """ConvTranspose2d(cin, nf, 2, 2) (diffusion_utilities.py:86) of x [B,Hin,Hin,cin] into y [B,2Hin,2Hin,nf]."""
        nf = self.nf
        if self.x16:
            lib().cdm_convT2x2_fwd_x16(x.p, B, Hin, Hin, cin, x.ld, _p(self.pk[name + ".wt_x"]),
                                       self._slot(ws, src_slot), self._wamax(name + ".wt"), _p(P[name + ".bias"]),
                                       _p(y), nf, nf, self._slot(ws, dst_slot), self.nterm, s)
        else:
            lib().cdm_convT2x2_fwd(x.p, B, Hin, Hin, cin, x.ld, _p(self.pk[name + ".wt"]), _p(P[name + ".bias"]),
                                   _p(y), nf, nf, self._slot(ws, dst_slot), s)

    def _conv_bn_fwd(self, ws, P, l: LayerSpec, s, x):
        lb = lib()
        B, S = ws.B, l.S
        src = ws.src[l.name]
        y = ws.y[l.name]
        st = ws.bn[l.name]
        npix = B * S * S
        if ws.train:
            if l.cin == 1:
                lb.cdm_conv3x3_cin1_fwd(_p(x), B, S, S, _p(self.pk[l.name + ".wpk"]), _p(P[l.b]), _p(y), l.cout,
                                        l.cout, 0, None, s)
                ymm_p, ymm_ld = ws.ymm_of(l) if (l.name in ws.fused_fwd and self.h3) else (None, 0)
                lb.cdm_reduce_stats_mm(_p(y), l.cout, B, S * S, l.cout, CHUNK, _p(ws.slab), ymm_p, ymm_ld, s)
                ntiles = B * _cdiv(S * S, CHUNK)
            else:
                yslot = self._slot(ws, "y:" + l.name) if l.name in ws.fused else None
                src, pre = self._src_pre(ws, l)
                ymm = ws.ymm_of(l) if (l.name in ws.fused_fwd and self.h3) else None
                self.conv3x3(l.name + ".wpk", src.p, B, S, l.cin, src.ld, _p(P[l.b]), _p(y), l.cout, l.cout, 0,
                             _p(ws.slab), l.cout, l.kc, s, amax_x=self._src_slot(ws, l), amax_y=yslot, pre=pre,
                             ymm=ymm, dt=self._fwd_dt(ws, l, pre))
                ntiles = _cdiv(npix, CHUNK)
            bn = l.bn
            nparts = fold(ws, _p(ws.slab), ntiles, 2, l.cout, s)
            fused_fwd = l.name in ws.fused_fwd
            ymm_p, ymm_ld = ws.ymm_of(l) if (fused_fwd and self.h3) else (None, 0)
            if ws.frozen:
                lb.cdm_bn_fwd_frozen(l.cout, _p(P[bn + ".weight"]), _p(P[bn + ".bias"]), _p(P[bn + ".running_mean"]),
                                     _p(P[bn + ".running_var"]), BN_EPS, _p(st["mean"]), _p(st["invstd"]),
                                     _p(st["scale"]), _p(st["shift"]), ymm_p, ymm_ld,
                                     self._dst_slot(ws, l) if fused_fwd else None, s)
            else:
                lb.cdm_bn_fwd_finalize(_p(ws.dpart), nparts, 2, l.cout, float(npix), _p(P[bn + ".weight"]),
                                       _p(P[bn + ".bias"]), _p(P[bn + ".running_mean"]), _p(P[bn + ".running_var"]),
                                       _p(P[bn + ".num_batches_tracked"]), BN_MOM, BN_EPS, _p(st["mean"]),
                                       _p(st["invstd"]), _p(st["scale"]), _p(st["shift"]), ymm_p, ymm_ld,
                                       self._dst_slot(ws, l) if fused_fwd else None, s)
            if fused_fwd:
                return                    # z = relu(y s + t) is applied by the next conv's staging
            scale, shift, relu = st["scale"], st["shift"], APPLY_RELU
        else:
            kind = ws.dst_kind[l.name]
            dense = kind in ("dense", "plain")
            outp = ws.dst[l.name] if dense else Act(y, l.cout)
            dslot = self._dst_slot(ws, l) if dense else None
            if l.cin == 1:
                lb.cdm_conv3x3_cin1_fwd(_p(x), B, S, S, _p(self.pk[l.name + ".wpk_e"]),
                                        _p(self.pk[l.name + ".bpk_e"]), outp.p, outp.ld, l.cout, 1, dslot, s)
            elif not dense and self.fuses_eval(l, B):
                # the residual add / FiLM / MaxPool in the conv's epilogue: y is never written
                self._conv_eval_fused(ws, l, kind, x, s)
                return
            else:
                self.conv3x3(l.name + ".wpk_e", src.p, B, S, l.cin, src.ld, _p(self.pk[l.name + ".bpk_e"]), outp.p,
                             outp.ld, l.cout, EPI_RELU, None, 0, l.kc, s, amax_x=self._src_slot(ws, l),
                             amax_y=dslot)
            if dense:
                return
            scale, shift, relu = self._ones, self._zeros, 0
        # apply: z = relu(bn(y)) -> destination (dense / pool / film / resid)
        kind = ws.dst_kind[l.name]
        dst = ws.dst[l.name]
        C = l.cout
        am = self._dst_slot(ws, l)
        if kind == "dense" or kind == "plain":
            lb.cdm_norm_apply_fwd(relu, _p(y), C, B, S, S, C, _p(scale), _p(shift), 0, None, 0, None, 0, None, None,
                                  None, 0, dst.p, dst.ld, am, s)
        elif kind == "pool":
            lb.cdm_norm_apply_fwd(APPLY_POOL | relu, _p(y), C, B, S, S, C, _p(scale), _p(shift), 0, None, 0, None, 0,
                                  None, None, None, 0, dst.p, dst.ld, am, s)
        elif kind == "film":
            ce, te = ws.emb["contextembed2"], ws.emb["timeembed2"]
            lb.cdm_norm_apply_fwd(APPLY_FILM | relu, _p(y), C, B, S, S, C, _p(scale), _p(shift), 0, _p(ce),
                                  C if ws.c_rows > 1 else 0, _p(te), C if ws.t_rows > 1 else 0, None, None, None, 0,
                                  dst.p, dst.ld, am, s)
        elif kind == "resid" and self.cp > 1:
            sc_w, sc_b, split = ws.sc_pending
            lb.cdm_norm_apply_fwd_resid_c(relu, _p(y), C, B, S, S, C, _p(scale), _p(shift), _p(x), self.cp, self.cimg,
                                          _p(sc_w), _p(sc_b), split, dst.p, dst.ld, am, s)
        elif kind == "resid":
            sc_w, sc_b, split = ws.sc_pending
            lb.cdm_norm_apply_fwd(APPLY_RESID | relu, _p(y), C, B, S, S, C, _p(scale), _p(shift), 0, None, 0, None,
                                  0, _p(x), _p(sc_w), _p(sc_b), split, dst.p, dst.ld, am, s)
        else:
            raise AssertionError(kind)

    def fuses_eval(self, l: "LayerSpec", B: int) -> bool:
        """Eval forward of a pool / FiLM / residual layer with its output transform in the LDS-halo conv's epilogue
        (cdm_conv3x3_fwd_x16_fused: 32^2 / 64^2 maps, 16-bit arithmetics); $CDM_FUSE_EVAL=0 keeps the apply kernel."""
        return (self.fuse_eval and l.cin > 1 and l.kc == 16 and l.S in (32, 64) and l.cout % 128 == 0
                and self.halo_addressable(B, l.S) and not (self.cp > 1 and l.name == "init_conv.conv2"))

    def _conv_eval_fused(self, ws, l: "LayerSpec", kind: str, x, s):
        lb = lib()
        B, S, C = ws.B, l.S, l.cout
        src = ws.src[l.name]
        dst = ws.dst[l.name]
        key = l.name + ".wpk_e"
        amax_x = self._src_slot(ws, l)
        if self.h3 and amax_x is None:
            amax_x = _p(self._amax)
            lb.cdm_amax_f32(src.p, B * S * S, l.cin, src.ld, amax_x, 0, s)
        sc_x = sc_w = sc_b = fa = fb = None
        split = fan = fbn = 0
        if kind == "resid":
            code = 1
            sc_w_t, sc_b_t, split = ws.sc_pending
            sc_x, sc_w, sc_b = _p(x), _p(sc_w_t), _p(sc_b_t)
        elif kind == "film":
            code = 2
            fa, fb = _p(ws.emb["contextembed2"]), _p(ws.emb["timeembed2"])
            fan, fbn = (C if ws.c_rows > 1 else 0), (C if ws.t_rows > 1 else 0)
        else:
            assert kind == "pool", kind
            code = 3
        lb.cdm_conv3x3_fwd_x16_fused(src.p, B, S, S, l.cin, src.ld, _p(self.pk[key + "_x"]), amax_x,
                                     self._wamax(key), _p(self.pk[l.name + ".bpk_e"]), dst.p, dst.ld, C, l.kc,
                                     self._dst_slot(ws, l), code, sc_x, sc_w, sc_b, split, fa, fan, fb, fbn,
                                     self.nterm, s)

    def _gn_fwd(self, ws, P, name, y: Act, B, S, C, st, stats_from_conv, stream):
        lb = lib()
        nchunks = _cdiv(S * S, CHUNK)
        if not stats_from_conv:
            lb.cdm_reduce_stats(y.p, y.ld, B, S * S, C, CHUNK, _p(ws.slab), stream)
        cpg = C // GN_GROUPS
        lb.cdm_gn_fwd_finalize(_p(ws.slab), B, nchunks, 2, C, GN_GROUPS, float(S * S * cpg), _p(P[name + ".weight"]),
                               _p(P[name + ".bias"]), GN_EPS, _p(st["mean"]), _p(st["invstd"]), _p(st["scale"]),
                               _p(st["shift"]), stream)

    # ------------------------------------------------------------------------------------------
    # backward (train mode workspaces only)
    # ------------------------------------------------------------------------------------------
    def backward(self, ws: "Workspace", P, deps: torch.Tensor, G: Dict[str, torch.Tensor], stream: int,
                 out3_bias_done: bool = False, on_stage=None, dx: Optional[torch.Tensor] = None,
                 dt: Optional[torch.Tensor] = None, dc: Optional[torch.Tensor] = None):
        """deps [B,H,W] = dL/d eps.  Writes (assigns) every parameter gradient into G[name].

        Optional input gradients (the module API under autograd, ContextUnet.py:42-60): dx [B,H,W] = dL/dx (the
        image), dt [rows_t] = dL/dt, dc [rows_c, n_cfeat] = dL/dc.  A t or c broadcast over the batch (one row) gets
        its embedding gradients summed over the samples.

        ``on_stage(name)`` is called (on the host, in stream order) as soon as the gradients of a stage
        are final: "out", "up2", "up1", "up0emb", "down2", "down1", "init" — used to start the
        data-parallel all-reduce of that stage while the rest of the backward runs."""
        hook = on_stage or (lambda name: None)
        assert ws.train, "backward needs a train-mode workspace"
        lb = lib(); s = stream
        nf, H, B = self.nf, self.H, ws.B
        H1, H2 = H // 2, H // 4
        P0, P1, P2 = B * H * H, B * H1 * H1, B * H2 * H2
        # ---------------- out.3 (nf -> 1) ----------------
        if self.cp > 1:
            gO = self._out3_bwd_c(ws, deps, G, s)
        else:
            R = cout1_band_rows(B, H)
            if ws.zO_fused:
                lb.cdm_conv3x3_cout1_wgrad_gn(_p(deps), _p(ws.yO), nf, B, H, H, nf, _p(ws.gnO["scale"]),
                                              _p(ws.gnO["shift"]), -R, _p(ws.slab), s)
            else:
                lb.cdm_conv3x3_cout1_wgrad(_p(deps), _p(ws.zO), nf, B, H, H, nf, -R, _p(ws.slab), s)
            S = fold(ws, _p(ws.slab), B * H // R, 9, nf, s)
            lb.cdm_slab_sum_all(_p(ws.dpart), S, 9, 0, 9, nf, _p(G["out.3.weight"]), 1, 9, 0, s)
            if not out3_bias_done:
                _sum_into(deps, G["out.3.bias"], ws, s)
            gO = ws.G0
            lb.cdm_conv3x3_cout1_dgrad(_p(deps), B, H, H, nf, _p(P["out.3.weight"]), _p(gO), nf, s)
        # ---------------- out.1 GroupNorm + ReLU ----------------
        dyO = ws.D0
        dslot = self._slot(ws, "dy:out.0")
        self._gn_bwd(ws, P, "out.1", "out.0.bias", Act(gO, nf), 0, Act(ws.yO, nf), B, H, nf, ws.gnO, None, 0,
                     Act(dyO, nf), G, s, amax=dslot)
        # ---------------- out.0 conv (2nf -> nf) ----------------
        self._wgrad3x3(ws, Act(dyO, nf), ws.catO, B, H, 2 * nf, nf, G["out.0.weight"], s, amax_dy=dslot,
                       amax_x=self._slot(ws, "catO"))
        self.conv3x3("out.0.wdg", _p(dyO), B, H, nf, nf, None, ws.dcatO.p, ws.dcatO.ld, 2 * nf, 0, None, 0,
                     self.kc_out0, s, amax_x=dslot,
                     amax_y=self._slot(ws, ws.out0_g_key) if ws.out0_g_key else None)
        hook("out")
        # ---------------- up2 blocks ----------------
        self._chain_bwd(ws, P, self.layers[14:18], G, s)
        # convT2 (2nf@H1 -> nf@H): grad wrt its output sits in ws.gT2
        self._convT_bwd(ws, P, "up2.model.0", Act(ws.gT2, nf), ws.catU2, B, H1, 2 * nf, nf, ws.dcatU2, G, s)
        hook("up2")
        # ---------------- up1 blocks (last one carries FiLM2) ----------------
        self._chain_bwd(ws, P, self.layers[10:14], G, s)
        self._convT_bwd(ws, P, "up1.model.0", Act(ws.gT1, nf), ws.catU1, B, H2, 4 * nf, nf, ws.dcatU1, G, s)
        hook("up1")
        # ---------------- up0: GroupNorm + ReLU + FiLM1 ----------------
        c0 = 2 * nf
        rows_c, rows_t = ws.c_rows, ws.t_rows
        self._gn_bwd(ws, P, "up0.1", "up0.0.bias", ws.dcatU1.sl(0, c0), 2, Act(ws.y0, c0), B, H2, c0, ws.gn0,
                     ws.emb["contextembed1"], c0 if rows_c > 1 else 0, Act(ws.D2, c0), G, s,
                     film_out=(ws.d_emb["contextembed1"], ws.d_emb["timeembed1"]))
        # up0 weight: dW[ci][(ij,co)] = sum_n hv[n][ci] dy0[n][(ij,co)]  -> [ci][co][ij]
        KN = self.KK0 * c0
        if self.up0_large:
            # dy0 [B][ij][co] -> [B][co][ij]: the K order of W[ci][(co, ij)] (134 MB at config 5, not the weights)
            lb.cdm_transpose_batched(_p(ws.D2), B, self.KK0, c0, _p(ws.up0T), s)
            if B <= 16 and c0 % 64 == 0:
                lb.cdm_up0_wgrad(_p(ws.hv), B, c0, _p(ws.D2), self.KK0, _p(G["up0.0.weight"]), s)
                # input gradient over W in place (VALU, W read once): per-K-range partials folded over the splits
                sp = lb.raw("cdm_up0_dgrad_splits")(c0, self.KK0)
                lb.cdm_up0_dgrad(_p(ws.up0T), B, c0, _p(P["up0.0.weight"]), self.KK0, _p(ws.slab), s)
                lb.cdm_slab_reduce(_p(ws.slab), sp, B, c0, _p(ws.dhv), c0, 0, 1, c0, 0, 1.0, s)
                a_dy = None
            else:
                sp = lb.raw("cdm_gemm_splits")(B, 1)
                lb.cdm_gemm_tn_f32(_p(ws.hv), c0, c0, B, _p(ws.up0T), KN, KN, 1, _p(ws.slab), s)
                lb.cdm_slab_reduce(_p(ws.slab), sp, c0, KN, _p(G["up0.0.weight"]), KN, 0, 1, 0, 0, 1.0, s)
                wT = self.pk["up0.WT"] = self._buf("up0.WT", (KN, c0))
                lb.cdm_transpose(_p(P["up0.0.weight"]), c0, KN, _p(wT), s)
                a_dy, w_t = ws.up0T, wT
        else:
            sp = lb.raw("cdm_gemm_splits")(B, 1)
            lb.cdm_gemm_tn_f32(_p(ws.hv), c0, c0, B, _p(ws.D2), KN, KN, 1, _p(ws.slab), s)
            if sp == 1:   # [ci][ij][co] -> [ci][co][ij]: a batched tiled transpose
                lb.cdm_transpose_batched(_p(ws.slab), c0, self.KK0, c0, _p(G["up0.0.weight"]), s)
            else:
                lb.cdm_slab_reduce(_p(ws.slab), sp, c0, KN, _p(G["up0.0.weight"]), KN, 1, self.KK0, c0, 0, 1.0, s)
            a_dy, w_t = ws.D2, self.pk["up0.wtT"]
        # dhv[n][ci] = sum_k dy0[n][k] W[ci][k] over k = (ij, co) or (co, ij) (large)   (split-K over 16*16*2nf)
        if a_dy is not None:
            want = max(1, min(64, _cdiv(1024, _cdiv(B, 128) * _cdiv(c0, 128))))
            sp = lb.raw("cdm_gemm_splits")(KN, want)
            lb.cdm_gemm_f32(_p(a_dy), KN, B, KN, _p(w_t), c0, c0, _p(ws.dhv), c0, None, 1, 0, sp,
                            _p(ws.slab), s)
            if sp > 1:
                lb.cdm_slab_reduce(_p(ws.slab), sp, B, c0, _p(ws.dhv), c0, 0, 1, c0, 0, 1.0, s)
        # to_vec: d2 grad += dhv * gelu'(hpre) / (h/4)^2
        d2g = ws.dcatU1.sl(2 * nf, 2 * nf)
        lb.cdm_avgpool_gelu_bwd(_p(ws.dhv), _p(ws.hpre), B, H2 * H2, c0, d2g.p, d2g.ld, s)
        # ---------------- embeddings ----------------
        d = ws._mlp
        for k, m in enumerate(MLPS):
            md = d.m[k]
            dout = ws.d_emb[m]
            if md.rows == 1 and B > 1:          # t / c broadcast over the batch: one embedding row, sums over samples
                E = dout.shape[1]
                lb.cdm_col_sum(_p(dout), B, E, _p(ws.d_emb_row[m]), 0, s)
                dout = ws.d_emb_row[m]
            md.dout = _p(dout); md.dpre = _p(ws.emb_dpre[m])
            md.dw1 = _p(G[m + ".model.0.weight"]); md.db1 = _p(G[m + ".model.0.bias"])
            md.dw2 = _p(G[m + ".model.2.weight"]); md.db2 = _p(G[m + ".model.2.bias"])
        lb.cdm_embed_bwd(ctypes_addr(d), s)
        for dv, (ma, mb), rows, in_dim in ((dt, ("timeembed1", "timeembed2"), ws.t_rows, 1),
                                           (dc, ("contextembed1", "contextembed2"), ws.c_rows, self.ncf)):
            if dv is not None:
                lb.cdm_embed_input_grad(_p(ws.emb_dpre[ma]), _p(P[ma + ".model.0.weight"]), 2 * nf,
                                        _p(ws.emb_dpre[mb]), _p(P[mb + ".model.0.weight"]), nf, rows, in_dim, _p(dv), s)
        hook("up0emb")
        # ---------------- down2, down1, init ----------------
        self._chain_bwd(ws, P, self.layers[6:10], G, s)
        hook("down2")
        self._chain_bwd(ws, P, self.layers[2:6], G, s)
        hook("down1")
        self._chain_bwd(ws, P, self.layers[0:2], G, s)
        if dx is not None:
            if self.cp > 1:
                self._image_grad_c(ws, dx, s)
            else:
                self._image_grad(ws, P, dx, s)
        hook("init")

    def _out3_bwd_c(self, ws, deps: torch.Tensor, G, s: int):
        """out.3 = Conv2d(n_feat, in_channels > 1) backward on the general kernels; deps = dL/d eps, NHWC [B*H*W, cp] with
        zero padding channels.  Returns the gradient wrt zO = relu(GN(yO)) (ws.G0)."""
        lb = lib()
        nf, H, B, cp, C = self.nf, self.H, ws.B, self.cp, self.cimg
        zslot = self._slot(ws, "zO")
        gw = self._buf("out.3.gwpad", (cp, nf, 3, 3))
        self._wgrad3x3(ws, Act(deps, cp), Act(ws.zO, nf), B, H, nf, cp, gw, s, amax_x=zslot)
        G["out.3.weight"].copy_(gw[:C])
        gb = self._buf("out.3.gbpad", (cp,))
        lb.cdm_reduce_sum(_p(deps), cp, B, H * H, cp, CHUNK, _p(ws.slab), s)
        nparts = fold(ws, _p(ws.slab), B * _cdiv(H * H, CHUNK), 1, cp, s)
        lb.cdm_slab_sum_all(_p(ws.dpart), nparts, 1, 0, 1, cp, _p(gb), 0, 1, 0, s)
        G["out.3.bias"].copy_(gb[:C])
        gO = ws.G0
        self.conv3x3("out.3.wdg", _p(deps), B, H, cp, cp, None, _p(gO), nf, nf, 0, None, 0, conv_kc(cp, nf), s)
        return gO

    def _image_grad_c(self, ws, dx: torch.Tensor, s: int):
        """dL/dx for in_channels > 1 (NHWC [B*H*W, cp]): init_conv.conv1's input gradient (its dgrad, already in
        ws.dgrad_dst) plus the random 1x1 shortcut's, dx[p][k] += sum_n g_res[p][n] w[n][k] (one GEMM)."""
        lb = lib()
        nf, H, B, cp, C = self.nf, self.H, ws.B, self.cp, self.cimg
        l = self.layers[0]
        P0 = B * H * H
        gd = ws.dgrad_dst[l.name]
        dx.view(P0, cp).copy_(gd.buf.view(-1)[: P0 * gd.ld].view(P0, gd.ld)[:, :cp])
        sc_w, _, split = ws.sc_pending
        assert split >= B, "input gradients with two shortcut draws (CFG halves) are not a module-call form"
        wpad = self._buf("sc.wpad", (nf, cp))
        wpad[:, C:].zero_(); wpad[:, :C].copy_(sc_w[: nf * C].view(nf, C))
        gres = ws.gout["init_conv.conv2"]
        sp = lib().raw("cdm_gemm_splits")(nf, 1)
        lb.cdm_gemm_f32(gres.p, gres.ld, P0, nf, _p(wpad), cp, cp, _p(dx), cp, None, 1, EPI_ACCUM, sp, _p(ws.slab), s)

    def _image_grad(self, ws, P, dx: torch.Tensor, s: int):
        """dL/dx of the image (ResidualConvBlock(1, nf, is_res) at diffusion_utilities.py:45-55 under autograd):
        init_conv.conv1's input gradient (the tap-flipped 3x3 conv over its BatchNorm + ReLU backward, applied while
        reading g and y) plus the random 1x1 shortcut's (sum_c w[c] * grad of the block output).  Runs after the init
        conv's backward, whose BatchNorm coefficients ws.coef still hold."""
        l = self.layers[0]
        C, B, H = l.cout, ws.B, self.H
        st, co = ws.bn[l.name], ws.coef
        g = ws.gout[l.name]
        gres = ws.gout["init_conv.conv2"]
        sc_w, _, split = ws.sc_pending
        if self.fuse_cin1_bwd:
            lib().cdm_conv3x3_cin1_dgrad(g.p, g.ld, _p(ws.y[l.name]), C, _p(st["scale"]), _p(st["shift"]),
                                         _p(st["mean"]), _p(st["invstd"]), _p(co[0]), _p(co[1]), _p(co[2]),
                                         _p(P[l.w]), gres.p, gres.ld, _p(sc_w), split, B, H, H, C, _p(dx), s)
        else:                                   # dy1 was written by cdm_norm_apply_bwd
            dy = ws.dy[l.name]
            lib().cdm_conv3x3_cin1_dgrad(dy.p, dy.ld, None, 0, None, None, None, None, None, None, None, _p(P[l.w]),
                                         gres.p, gres.ld, _p(sc_w), split, B, H, H, C, _p(dx), s)

    def _chain_bwd(self, ws, P, layers, G, s):
        for l in reversed(layers):
            self._conv_bn_bwd(ws, P, l, G, s)

    def _conv_bn_bwd(self, ws, P, l: LayerSpec, G, s):
        lb = lib()
        B, S, C = ws.B, l.S, l.cout
        kind = ws.dst_kind[l.name]
        g = ws.gout[l.name]
        y = ws.y[l.name]
        st = ws.bn[l.name]
        mode = {"dense": 0, "plain": 0, "resid": 0, "pool": 1, "film": 2}[kind]
        film_a, film_an = None, 0
        if mode == 2:
            film_a, film_an = ws.emb["contextembed2"], (C if ws.c_rows > 1 else 0)
        HWp = (S // 2) * (S // 2) if mode == 1 else S * S
        nch = _cdiv(HWp, CHUNK)
        co = ws.coef
        bn = l.bn
        if l.name in ws.sums_by:
            # the sums came with the consumer's weight gradient (PreBnReluSums): one partial per split
            assert mode == 0
            nparts = fold(ws, _p(ws.sums), ws.sums_sp[l.name], 5, C, s)
        else:
            assert l.name not in ws.act16, "bf16 activations need the fused BN-backward sums"
            lb.cdm_norm_bwd_reduce(mode, g.p, g.ld, _p(y), C, B, S, S, C, _p(st["scale"]), _p(st["shift"]), 0,
                                   _p(st["mean"]), _p(st["invstd"]), 0, 1, _p(film_a), film_an, CHUNK, _p(ws.slab), s)
            if mode == 2:  # FiLM2 sums -> d cemb2 / d temb2 (per sample)
                lb.cdm_slab_sum_nc(_p(ws.slab), B, nch, 5, 2, C, _p(ws.d_emb["contextembed2"]), s)
                lb.cdm_slab_sum_nc(_p(ws.slab), B, nch, 5, 3, C, _p(ws.d_emb["timeembed2"]), s)
            nparts = fold(ws, _p(ws.slab), B * nch, 5, C, s)
        fin = lb.cdm_bn_bwd_finalize_frozen if ws.frozen else lb.cdm_bn_bwd_finalize
        fin(_p(ws.dpart), nparts, C, float(B * S * S), _p(P[bn + ".weight"]), _p(st["invstd"]), _p(G[bn + ".weight"]),
            _p(G[bn + ".bias"]), _p(co[0]), _p(co[1]), _p(co[2]), _p(G[l.b]), s)
        gslot = self._dgrad_amax_slot(ws, l)
        if l.name in ws.fused:
            # dy = bn_bwd(g, y) inside the staging of both convs; its scale from a bound on max|dy|
            dslot = self._slot(ws, "dy:" + l.name)
            if self.h3:
                lb.cdm_bn_bwd_amax_bound(C, _p(co[0]), _p(co[1]), _p(co[2]), _p(st["mean"]), _p(st["invstd"]),
                                         self._slot(ws, "g:" + l.name), self._slot(ws, "y:" + l.name), dslot, s)
            coef = (_p(st["scale"]), _p(st["shift"]), _p(st["mean"]), _p(st["invstd"]), _p(co[0]), _p(co[1]),
                    _p(co[2]))
            src, pre = self._src_pre(ws, l)
            sp = wgrad_splits(B * S * S, C, 9 * l.cin)
            # dgrad first: it writes the producer's g, which the weight gradient's producer sums read
            dgd = ws.dgrad_dst[l.name]
            key = l.name + ".wdg"
            own16 = 1 if l.name in ws.act16 else 0
            if ws.dyo is not None:
                if self.dy_pass:
                    # bf16 arithmetic: dy by its own elementwise pass, then the dgrad on the LDS-halo forward schedule
                    # (halo two chunks ahead, one barrier per chunk) — the fused BN-backward staging has no room for it
                    lb.cdm_bn_bwd_dy(g.p, g.ld, _p(y), C, B * S * S, C, *coef, _p(ws.dyo), g.ld, own16 | (own16 << 1), s)
                    self.conv3x3(key, _p(ws.dyo), B, S, C, g.ld, None, dgd.p, dgd.ld, l.cin,
                                 EPI_ACCUM if ws.dgrad_accum[l.name] else 0, None, 0, l.kc, s, amax_y=gslot,
                                 dt=own16 | self._dgrad_out16(ws, l))
                else:
                    # the dgrad stores dy; the weight gradient stages it (no BN backward there)
                    lb.cdm_conv3x3_dgrad_x16_bnbwd_dy(g.p, g.ld, _p(y), C, *coef, B, S, S, C, _p(self.pk[key + "_x"]),
                                                      dslot, self._wamax(key), dgd.p, dgd.ld, l.cin,
                                                      EPI_ACCUM if ws.dgrad_accum[l.name] else 0, gslot, _p(ws.dyo),
                                                      self.nterm, own16 | self._dgrad_out16(ws, l), s)
                nul = (None,) * 7
                if pre is None:
                    lb.cdm_conv3x3_wgrad_x16_ex(_p(ws.dyo), g.ld, None, 0, *nul, C, src.p, B, S, S, l.cin, src.ld, None,
                                                None, None, 0, None, None, None, dslot, self._src_slot(ws, l), sp,
                                                _p(ws.slab), self.nterm, own16, s)
                else:
                    lb.cdm_conv3x3_wgrad_x16_ex(_p(ws.dyo), g.ld, None, 0, *nul, C, src.p, B, S, S, l.cin, src.ld,
                                                pre[0], pre[1], *self._producer_sums(ws, l, sp), dslot,
                                                self._src_slot(ws, l), sp, _p(ws.slab), self.nterm,
                                                own16 | self._prod16(ws, l), s)
                lb.cdm_slab_reduce(_p(ws.slab), sp, C, 9 * l.cin, _p(G[l.w]), 9 * l.cin, 1, 9, l.cin, 0, 1.0, s)
                return
            lb.cdm_conv3x3_dgrad_x16_bnbwd(g.p, g.ld, _p(y), C, *coef, B, S, S, C, _p(self.pk[key + "_x"]), dslot,
                                           self._wamax(key), dgd.p, dgd.ld, l.cin,
                                           EPI_ACCUM if ws.dgrad_accum[l.name] else 0, gslot, self.nterm,
                                           own16 | self._dgrad_out16(ws, l), s)
            if pre is None:
                lb.cdm_conv3x3_wgrad_x16_bnbwd(g.p, g.ld, _p(y), C, *coef, C, src.p, B, S, S, l.cin, src.ld, dslot,
                                               self._src_slot(ws, l), sp, _p(ws.slab), self.nterm, own16, s)
            else:
                lb.cdm_conv3x3_wgrad_x16_ex(g.p, g.ld, _p(y), C, *coef, C, src.p, B, S, S, l.cin, src.ld, pre[0],
                                            pre[1], *self._producer_sums(ws, l, sp), dslot, self._src_slot(ws, l), sp,
                                            _p(ws.slab), self.nterm, own16 | self._prod16(ws, l), s)
            lb.cdm_slab_reduce(_p(ws.slab), sp, C, 9 * l.cin, _p(G[l.w]), 9 * l.cin, 1, 9, l.cin, 0, 1.0, s)
            return
        if l.cin == 1 and mode == 0 and self.fuse_cin1_bwd:
            # init_conv.conv1: only a weight gradient (the input needs none); its BN backward runs while that kernel
            # reads g and y (bit-identical dy, never written)
            lb.cdm_conv3x3_cin1_wgrad_bnbwd(g.p, g.ld, _p(y), C, _p(st["scale"]), _p(st["shift"]), _p(st["mean"]),
                                            _p(st["invstd"]), _p(co[0]), _p(co[1]), _p(co[2]), _p(ws.x_in), B, S, S,
                                            C, CHUNK, _p(ws.slab), s)
            nparts = fold(ws, _p(ws.slab), B * _cdiv(S * S, CHUNK), 10, C, s)
            lb.cdm_slab_sum_all(_p(ws.dpart), nparts, 10, 0, 9, C, _p(G[l.w]), 1, 9, 0, s)
            return
        dy = ws.dy[l.name]
        dslot = self._slot(ws, "dy:" + l.name) if l.cin > 1 else None
        lb.cdm_norm_apply_bwd(mode, g.p, g.ld, _p(y), C, B, S, S, C, _p(st["scale"]), _p(st["shift"]), 0,
                              _p(st["mean"]), _p(st["invstd"]), 0, 1, _p(film_a), film_an, _p(co[0]), _p(co[1]),
                              _p(co[2]), 0, dy.p, dy.ld, dslot, s)
        src, pre = self._src_pre(ws, l)
        if l.cin == 1:
            lb.cdm_conv3x3_cin1_wgrad(dy.p, dy.ld, _p(ws.x_in), B, S, S, C, CHUNK, _p(ws.slab), s)
            nparts = fold(ws, _p(ws.slab), B * _cdiv(S * S, CHUNK), 10, C, s)
            lb.cdm_slab_sum_all(_p(ws.dpart), nparts, 10, 0, 9, C, _p(G[l.w]), 1, 9, 0, s)
            return
        dgd = ws.dgrad_dst[l.name]
        # dgrad first (it writes the producer's g, read by the producer sums of the weight gradient below)
        self.conv3x3(l.name + ".wdg", dy.p, B, S, C, dy.ld, None, dgd.p, dgd.ld, l.cin,
                     EPI_ACCUM if ws.dgrad_accum[l.name] else 0, None, 0, l.kc, s, amax_x=dslot, amax_y=gslot,
                     dt=self._dgrad_out16(ws, l))
        pad0 = l is self.layers[0] and self.cp > self.cimg      # the init conv's zero image-channel columns
        gW = self._buf("init.gwpad", (C, self.cp, 3, 3)) if pad0 else G[l.w]
        self._wgrad3x3(ws, dy, src, B, S, l.cin, C, gW, s, amax_dy=dslot, amax_x=self._src_slot(ws, l), pre=pre,
                       sums_of=l)
        if pad0:
            G[l.w].copy_(gW[:, :self.cimg])

    def _src_pre(self, ws, l: "LayerSpec"):
        """(input activation, BN-ReLU transform or None) of conv l in train mode: a fused producer hands over its
        pre-norm output y and its (scale, shift) instead of z."""
        i = self.layers.index(l)
        if i > 0 and self.layers[i - 1].name in ws.fused_fwd:
            p = self.layers[i - 1]
            st = ws.bn[p.name]
            return Act(ws.y[p.name], p.cout), (_p(st["scale"]), _p(st["shift"]))
        return ws.src[l.name], None

    # bf16 activation storage (C4): dtype bits of the conv launches around layer l ---------------------------------
    def _prod16(self, ws, l: "LayerSpec") -> int:
        """2 when conv l's input is the bf16 pre-norm output of a fused producer (its staging applies BN-ReLU), else 0."""
        i = self.layers.index(l)
        return 2 if (i > 0 and self.layers[i - 1].name in ws.act16 and self.layers[i - 1].name in ws.fused_fwd) else 0

    def _fwd_dt(self, ws, l: "LayerSpec", pre) -> int:
        """forward conv l: bit 0 its source is a bf16 y (BN-ReLU staged), bit 1 its y is stored as bf16."""
        src16 = 1 if (pre is not None and self._prod16(ws, l)) else 0
        return src16 | (2 if l.name in ws.act16 else 0)

    def _dgrad_out16(self, ws, l: "LayerSpec") -> int:
        """2 when the input gradient conv l writes (the gradient of its producer's output) is stored as bf16."""
        i = self.layers.index(l)
        if i == 0 or ws.dgrad_accum.get(l.name, False):
            return 0
        p = self.layers[i - 1]
        return 2 if (p.name in ws.act16 and ws.gout[p.name].buf.data_ptr() == ws.dgrad_dst[l.name].buf.data_ptr()) else 0

    def _dgrad_amax_slot(self, ws, l: "LayerSpec"):
        """Slot that receives max|dgrad output| of layer l: the grad wrt a ConvT output (h3 ConvT backward) or
        the grad g of a fused layer (its dy bound)."""
        if l.name in self._CONVT_GRAD_PRODUCERS:
            return self._slot(ws, "gT:" + l.name)
        key = ws.g_amax_key.get(l.name)
        return self._slot(ws, key) if key else None

    # the dgrads that write the gradient wrt a ConvT output (gT1 / gT2) also record its max for the h3 ConvT bwd
    _CONVT_GRAD_PRODUCERS = {"up1.model.1.conv1": "up1.model.0", "up2.model.1.conv1": "up2.model.0"}

    def _producer_sums(self, ws, l: "LayerSpec", sp: int):
        """(x_g, ldxg, x_mean, x_invstd, x_sums) for conv l's weight gradient: the BN-backward sums of its fused producer
        when they ride along (ws.sums_from), else all null."""
        pn = ws.sums_from.get(l.name)
        if pn is None:
            return None, 0, None, None, None
        g, st = ws.gout[pn], ws.bn[pn]
        ws.sums_sp[pn] = sp * 3 * (l.cout // 128)     # one partial per block: split x kernel row x co tile
        return g.p, g.ld, _p(st["mean"]), _p(st["invstd"]), _p(ws.sums)

    def _wgrad3x3(self, ws, dy: Act, x: Act, B, S, cin, cout, gW, s, amax_dy=None, amax_x=None, pre=None,
                  sums_of=None):
        lb = lib()
        sp = wgrad_splits(B * S * S, cout, 9 * cin)
        if pre is not None:        # X = relu(x s + t) of a fused producer (16-bit arithmetic, kernel-row weight gradient)
            sums = self._producer_sums(ws, sums_of, sp) if sums_of is not None else (None, 0, None, None, None)
            dt = 2 if (sums_of is not None and self._prod16(ws, sums_of)) else 0
            lb.cdm_conv3x3_wgrad_x16_ex(dy.p, dy.ld, None, 0, None, None, None, None, None, None, None, cout, x.p, B, S,
                                        S, cin, x.ld, pre[0], pre[1], *sums, amax_dy, amax_x, sp, _p(ws.slab),
                                        self.nterm, dt, s)
            lb.cdm_slab_reduce(_p(ws.slab), sp, cout, 9 * cin, _p(gW), 9 * cin, 1, 9, cin, 0, 1.0, s)
            return
        if S % 8:
            # the 16-bit weight-gradient GEMMs stage 8-pixel pieces of one image row: other widths take the fp32 GEMM
            lb.cdm_conv3x3_wgrad(dy.p, dy.ld, cout, x.p, B, S, S, cin, x.ld, sp, _p(ws.slab), s)
        elif self.x16:
            am = _p(self._amax)
            if self.h3 and amax_dy is None:
                amax_dy = am
                lb.cdm_amax_f32(dy.p, B * S * S, cout, dy.ld, amax_dy, 0, s)
            if self.h3 and amax_x is None:
                amax_x = am + 4
                lb.cdm_amax_f32(x.p, B * S * S, cin, x.ld, amax_x, 0, s)
            lb.cdm_conv3x3_wgrad_x16(dy.p, dy.ld, cout, x.p, B, S, S, cin, x.ld, amax_dy, amax_x, sp, _p(ws.slab),
                                     self.nterm, s)
        elif self.nterm:
            lb.cdm_conv3x3_wgrad_x3(dy.p, dy.ld, cout, x.p, B, S, S, cin, x.ld, sp, _p(ws.slab), self.nterm, s)
        else:
            lb.cdm_conv3x3_wgrad(dy.p, dy.ld, cout, x.p, B, S, S, cin, x.ld, sp, _p(ws.slab), s)
        # slab[z][co][tap*cin+ci] -> OIHW [co][ci][tap]
        lb.cdm_slab_reduce(_p(ws.slab), sp, cout, 9 * cin, _p(gW), 9 * cin, 1, 9, cin, 0, 1.0, s)

    def _convT_bwd(self, ws, P, name, gy: Act, x: Act, B, Hin, cin, cout, dx: Act, G, s):
        """ConvTranspose2d(cin, cout, 2, 2) backward; gy is the grad of its output [B, 2Hin, 2Hin, cout]."""
        lb = lib()
        Ho = 2 * Hin
        lb.cdm_reduce_sum(gy.p, gy.ld, B, Ho * Ho, cout, CHUNK, _p(ws.slab), s)
        nparts = fold(ws, _p(ws.slab), B * _cdiv(Ho * Ho, CHUNK), 1, cout, s)
        lb.cdm_slab_sum_all(_p(ws.dpart), nparts, 1, 0, 1, cout, _p(G[name + ".bias"]), 0, 1, 0, s)
        sp = wgrad_splits(B * Hin * Hin, cin, 4 * cout)
        x16 = self.x16
        if x16 and Hin % 8 == 0:
            prod = next(k for k, v in self._CONVT_GRAD_PRODUCERS.items() if v == name)
            a_gy = self._slot(ws, "gT:" + prod)
            a_x = self._slot(ws, {"up1.model.0": "catU1", "up2.model.0": "catU2"}[name])
            lb.cdm_convT2x2_wgrad_x16(x.p, B, Hin, Hin, cin, x.ld, gy.p, cout, gy.ld, a_x, a_gy, sp, _p(ws.slab),
                                      self.nterm, s)
        else:   # fp32 arithmetic, or an input grid whose width is not a multiple of 8 (the 16-bit GEMM's pieces)
            lb.cdm_convT2x2_wgrad(x.p, B, Hin, Hin, cin, x.ld, gy.p, cout, gy.ld, sp, _p(ws.slab), s)
        # slab[z][ci][ij*cout+co] -> [ci][co][ij]
        lb.cdm_slab_reduce(_p(ws.slab), sp, cin, 4 * cout, _p(G[name + ".weight"]), 4 * cout, 1, 4, cout, 0, 1.0, s)
        if self.x16:
            a_gy = self._slot(ws, "gT:" + next(k for k, v in self._CONVT_GRAD_PRODUCERS.items() if v == name))
            lb.cdm_convT2x2_dgrad_x16(gy.p, B, Hin, Hin, cout, gy.ld, _p(self.pk[name + ".wtT_x"]), a_gy,
                                      self._wamax(name + ".wtT"), dx.p, dx.ld, cin, 0, self.nterm, s)
        else:
            lb.cdm_convT2x2_dgrad(gy.p, B, Hin, Hin, cout, gy.ld, _p(self.pk[name + ".wtT"]), dx.p, dx.ld, cin, 0, s)

    def _gn_bwd(self, ws, P, name, bias_name, g: Act, mode, y: Act, B, S, C, st, film_a, film_an, dy: Act, G, s,
                film_out=None, amax=None):
        lb = lib()
        nch = _cdiv(S * S, CHUNK)
        cpg = C // GN_GROUPS
        lb.cdm_norm_bwd_reduce(mode, g.p, g.ld, y.p, y.ld, B, S, S, C, _p(st["scale"]), _p(st["shift"]), C,
                               _p(st["mean"]), _p(st["invstd"]), GN_GROUPS, cpg, _p(film_a), film_an, CHUNK,
                               _p(ws.slab), s)
        if film_out is not None:
            lb.cdm_slab_sum_nc(_p(ws.slab), B, nch, 5, 2, C, _p(film_out[0]), s)
            lb.cdm_slab_sum_nc(_p(ws.slab), B, nch, 5, 3, C, _p(film_out[1]), s)
        co = ws.gcoef
        lb.cdm_gn_bwd_finalize(_p(ws.slab), B, nch, C, GN_GROUPS, float(S * S * cpg), S * S, _p(P[name + ".weight"]),
                               _p(st["invstd"]), _p(co[0]), _p(co[1]), _p(co[2]), _p(co[3]), _p(co[4]), _p(co[5]), s)
        lb.cdm_col_sum3(_p(co[3]), _p(G[name + ".weight"]), _p(co[4]), _p(G[name + ".bias"]),
                        _p(co[5]) if bias_name is not None else None,
                        _p(G[bias_name]) if bias_name is not None else None, B, C, s)
        lb.cdm_norm_apply_bwd(mode, g.p, g.ld, y.p, y.ld, B, S, S, C, _p(st["scale"]), _p(st["shift"]), C,
                              _p(st["mean"]), _p(st["invstd"]), GN_GROUPS, cpg, _p(film_a), film_an, _p(co[0]),
                              _p(co[1]), _p(co[2]), C, dy.p, dy.ld, amax, s)


def _sum_into(x: torch.Tensor, out: torch.Tensor, ws, stream: int):
    """out[0] = sum(x) for a C=1 map: C=4 column partials over a [n/4, 4] view, then fold."""
    lb = lib()
    n = x.numel()
    assert n % 4 == 0
    nch = _cdiv(n // 4, CHUNK)
    scratch = ws.slab
    lb.cdm_reduce_sum(_p(x), 4, 1, n // 4, 4, CHUNK, _p(scratch), stream)
    part = scratch[4 * nch: 4 * nch + 4]
    S = fold(ws, _p(scratch), nch, 1, 4, stream)
    lb.cdm_slab_sum_all(_p(ws.dpart), S, 1, 0, 1, 4, _p(part), 0, 1, 0, stream)
    lb.cdm_col_sum(_p(part), 4, 1, _p(out), 0, stream)


def fold(ws, slab_ptr: int, ntiles: int, R: int, C: int, stream: int) -> int:
    """Stage-1 parallel fold of an fp32 partial slab [ntiles][R][C] into fp64 parts; returns #parts."""
    S = max(1, min(ntiles, max(1, 512 // _cdiv(C, 64)), ws.dpart.numel() // max(1, R * C)))
    lib().cdm_slab_colsum(slab_ptr, ntiles, R, C, _p(ws.dpart), S, stream)
    return S


def cout1_band_rows(B: int, H: int) -> int:
    """Rows per block of the out.3 weight-gradient band kernel: the largest divisor of H that still gives >= 1024
    blocks (B=256 at 64x64: 16 rows -> 1024 blocks)."""
    R = H
    while R > 1 and (B * H // R < 1024 or H % R):
        R -= 1
    return R


def wgrad_splits(K: int, M: int, N: int) -> int:
    """Split-K factor for a weight-gradient GEMM (M = C_out, N = 9 C_in for a 3x3 conv, K = pixels).

    3x3 convs with C_in, C_out % 128 == 0 run the kernel-row weight gradient: 3 (C_out/128) (C_in/128) blocks per split,
    one 512-thread block per CU at a time, all blocks equal work — so the grid is sized to whole rounds of 256 CUs
    (768 blocks): 228 splits gave 684 blocks = 2.67 rounds, whose last round ran a third empty (same-box A/B,
    profiles/r3_ab_wgrad_rounds.txt: C2 train step 53.04 -> 51.89 ms, C4 33.09 -> 32.12 ms).  Others: ~2048
    workgroups of the generic split GEMM."""
    if N % 9 == 0 and M % 128 == 0 and (N // 9) % 128 == 0 and os.environ.get("CDM_WGRAD_ROUNDS", "1") != "0":
        per = 3 * (M // 128) * ((N // 9) // 128)
        want = max(1, min(512, round(int(os.environ.get("CDM_WGRAD_BLOCKS", "768")) / per)))
        return lib().raw("cdm_gemm_splits")(K, want)
    tiles = _cdiv(M, 128) * _cdiv(N, 128)
    want = max(1, min(512, _cdiv(2048, tiles)))
    return lib().raw("cdm_gemm_splits")(K, want)


def ctypes_addr(obj):
    import ctypes
    return ctypes.addressof(obj)


class Workspace:
    """All device buffers for one batch size and mode (train keeps what backward needs)."""

    def __init__(self, eng: UNetEngine, B: int, train: bool, frozen: bool = False):
        self.eng, self.B, self.train = eng, B, train
        self.frozen = False          # set by each forward (eval-mode BatchNorm in a train-structured forward)
        self.zO_fused = False        # set by each forward: out.1's GroupNorm + ReLU applied inside out.3's kernels
        dev = eng.device
        nf, H, ncf = eng.nf, eng.H, eng.ncf
        H1, H2 = H // 2, H // 4
        P0, P1, P2 = B * H * H, B * H1 * H1, B * H2 * H2
        E = lambda *shape: torch.empty(*shape, device=dev, dtype=torch.float32)
        self.catO = Act(E(P0, 2 * nf), 2 * nf)
        self.catU2 = Act(E(P1, 2 * nf), 2 * nf)
        self.catU1 = Act(E(P2, 4 * nf), 4 * nf)
        self.eps = E(B, H, H) if eng.cp == 1 else E(P0, eng.cp)
        self.yT1 = E(P1, nf)
        self.yT2 = E(P0, nf)
        self.y0 = E(P2, 2 * nf)
        self.yO = E(P0, nf)
        # zO = relu(GN(yO)) only exists where out.3 cannot apply out.1 in its staging (537 MB at the bench shape)
        self.zO = E(P0, nf) if not eng.fuses_gn_out(train) else torch.empty(0, device=dev)
        self.hsum, self.hpre, self.hv = E(B, 2 * nf), E(B, 2 * nf), E(B, 2 * nf)
        self.c_zero = torch.zeros(B, ncf, device=dev)
        self.emb = {m: E(B, (2 if m.endswith("1") else 1) * nf) for m in MLPS}
        if train:
            self.emb_pre = {m: E(B, (2 if m.endswith("1") else 1) * nf) for m in MLPS}
            self.emb_h = {m: E(B, (2 if m.endswith("1") else 1) * nf) for m in MLPS}
            self.emb_dpre = {m: E(B, (2 if m.endswith("1") else 1) * nf) for m in MLPS}
            self.d_emb = {m: E(B, (2 if m.endswith("1") else 1) * nf) for m in MLPS}
            self.d_emb_row = {m: E(1, (2 if m.endswith("1") else 1) * nf) for m in MLPS}   # broadcast t / c
        self.gn0 = {k: E(B * 2 * nf) for k in ("mean", "invstd", "scale", "shift")}
        self.gnO = {k: E(B * nf) for k in ("mean", "invstd", "scale", "shift")}
        # per conv-BN layer: y (pre-norm), z destinations, BN coefficients
        L = eng.layers
        self.y, self.src, self.dst, self.dst_kind, self.bn = {}, {}, {}, {}, {}
        self._no_z = torch.empty(0, device=dev)
        z = {}
        for l in L:
            npx = B * l.S * l.S
            self.y[l.name] = E(npx, l.cout)
            self.bn[l.name] = {k: E(l.cout) for k in ("mean", "invstd", "scale", "shift")}
        names = [l.name for l in L]
        # destinations of each layer's activation output
        kinds = {}
        for i, l in enumerate(L):
            kinds[l.name] = "dense"
        kinds["init_conv.conv2"] = "resid"
        kinds["down1.model.1.conv2"] = "pool"
        kinds["down2.model.1.conv2"] = "pool"
        kinds["up1.model.2.conv2"] = "film"
        kinds["up2.model.2.conv2"] = "plain"
        self.dst_kind = kinds
        self.fused_fwd = {l.name for l in L if train and eng.fuses_bn_fwd(l, kinds[l.name], B)}
        for l in L:
            k = kinds[l.name]
            if k == "dense":
                # a fused producer's z is never materialised (the consumer stages relu(y s + t) itself)
                z[l.name] = Act(E(B * l.S * l.S, l.cout) if l.name not in self.fused_fwd else self._no_z, l.cout)
                self.dst[l.name] = z[l.name]
        self.dst["init_conv.conv2"] = self.catO.sl(nf, nf)
        self.dst["down1.model.1.conv2"] = self.catU2.sl(nf, nf)
        self.dst["down2.model.1.conv2"] = self.catU1.sl(2 * nf, 2 * nf)
        self.dst["up1.model.2.conv2"] = self.catU2.sl(0, nf)
        self.dst["up2.model.2.conv2"] = self.catO.sl(0, nf)
        # inputs of each conv
        prev = {names[i]: names[i - 1] for i in range(1, len(names))}
        for l in L:
            if l.name == "init_conv.conv1":
                self.src[l.name] = None
            elif l.name == "down1.model.0.conv1":
                self.src[l.name] = self.catO.sl(nf, nf)
            elif l.name == "down2.model.0.conv1":
                self.src[l.name] = self.catU2.sl(nf, nf)
            elif l.name == "up1.model.1.conv1":
                self.src[l.name] = Act(self.yT1, nf)
            elif l.name == "up2.model.1.conv1":
                self.src[l.name] = Act(self.yT2, nf)
            else:
                self.src[l.name] = self.dst[prev[l.name]]
        self.slab = E(self._slab_floats())
        # per fused layer: max / min keys of its pre-norm output ([2][n_fused][Cmax] int32, refilled every forward)
        self._ymm_idx = {n: i for i, n in enumerate(sorted(self.fused_fwd))}
        self._ymm_C = max([l.cout for l in L] + [1])
        self.ymm = torch.empty(2 * max(1, len(self.fused_fwd)) * self._ymm_C, dtype=torch.int32, device=dev)
        self.amax = torch.zeros(192, device=dev)  # h3 operand maxima, one slot per producer (UNetEngine._slot)
        self.aslot = {}
        self.dpart = torch.empty(10 * 32768 + 4096, device=dev, dtype=torch.float64)
        self.sc_pending = None
        if train:
            C4 = 4 * nf
            self.G0, self.D0 = E(P0, 2 * nf), E(P0, 2 * nf)
            self.G1, self.D1 = E(P1, 2 * nf), E(P1, 2 * nf)
            self.D2 = E(P2, 4 * nf)
            self.gT1, self.gT2 = self.G1, self.G0
            self.dcatO = Act(E(P0, 2 * nf), 2 * nf)
            self.dcatU2 = Act(E(P1, 2 * nf), 2 * nf)
            self.dcatU1 = Act(E(P2, 4 * nf), 4 * nf)
            self.dhv = E(B, 2 * nf)
            self.up0T = E(P2, 2 * nf) if eng.up0_large else None   # dy0 with (co, ij) order (large up0)
            self.coef = [E(C4) for _ in range(3)]
            self.gcoef = [E(B * C4) for _ in range(6)]
            # backward wiring: grad of each layer's output (gout), its dy buffer and dgrad destination
            self.gout, self.dy, self.dgrad_dst, self.dgrad_accum = {}, {}, {}, {}
            for l in L:
                Gb = self.G0 if l.S == H else self.G1
                Db = self.D0 if l.S == H else self.D1
                self.dy[l.name] = Act(Db, l.cout)
                k = kinds[l.name]
                if k == "resid":
                    self.gout[l.name] = self.dcatO.sl(nf, nf)
                elif k == "pool":
                    self.gout[l.name] = (self.dcatU2.sl(nf, nf) if l.name.startswith("down1")
                                         else self.dcatU1.sl(2 * nf, 2 * nf))
                elif k == "film":
                    self.gout[l.name] = self.dcatU2.sl(0, nf)
                elif k == "plain":
                    self.gout[l.name] = self.dcatO.sl(0, nf)
                else:
                    self.gout[l.name] = Act(Gb, l.cout)   # written by the next layer's dgrad
                # where this layer's dgrad (grad wrt its input) goes
                if l.name == "down1.model.0.conv1":
                    self.dgrad_dst[l.name], self.dgrad_accum[l.name] = self.dcatO.sl(nf, nf), True
                elif l.name == "down2.model.0.conv1":
                    self.dgrad_dst[l.name], self.dgrad_accum[l.name] = self.dcatU2.sl(nf, nf), True
                elif l.name in ("up1.model.1.conv1", "up2.model.1.conv1"):
                    self.dgrad_dst[l.name], self.dgrad_accum[l.name] = Act(Gb, l.cin), False
                elif l.cin > 1:
                    self.dgrad_dst[l.name], self.dgrad_accum[l.name] = Act(Gb, l.cin), False
            self._wire_fused_bn_bwd(eng, L, kinds)
            # the fused layers' dy (eng.dy_store): one buffer, rewritten by each fused layer's dgrad and read by its
            # weight gradient right after; g's row stride (fp32 size, bf16 dy use half)
            self.dyo = None
            if eng.dy_store and self.fused:
                self.dyo = E(max(B * l.S * l.S * self.gout[l.name].ld for l in L if l.name in self.fused))
            # producer BN-backward sums in the consumer's weight gradient: a fused (BN-ReLU staged) dense producer p
            # whose consumer c takes the kernel-row weight gradient with the X transform
            self.sums_from, self.sums_by, self.sums_sp = {}, {}, {}
            if eng.fuse_bn_sums:
                for i in range(1, len(L)):
                    p_, c_ = L[i - 1], L[i]
                    if p_.name in self.fused_fwd and kinds[p_.name] == "dense" and c_.cin % 128 == 0 \
                            and c_.cout % 128 == 0 and c_.S % 16 == 0:
                        self.sums_from[c_.name], self.sums_by[p_.name] = p_.name, c_.name
            nsum = max([wgrad_splits(B * L[i].S * L[i].S, L[i].cout, 9 * L[i].cin) * 3 * (L[i].cout // 128) * 5
                        * L[i].cin for i in range(len(L)) if L[i].name in self.sums_from] + [1])
            self.sums = E(nsum)
            # bf16 activations (C4): the fused chain's y and g (layers whose BN-ReLU apply runs in the next conv's
            # staging, C_in > 1; each has its BN-backward sums fused into the consumer's weight gradient and a private
            # gradient buffer, so every kernel reading them is one of the two templated conv kernels)
            self.act16 = set()
            if eng.act16 and not frozen:
                self.act16 = {l.name for l in L if l.name in self.fused_fwd and l.cin > 1 and l.name in self.sums_by
                              and l.name in self.fused and self.gout[l.name].off == 0}
        else:
            self.fused, self.g_amax_key, self.out0_g_key = set(), {}, None
            self.sums_from, self.sums_by, self.sums_sp = {}, {}, {}
            self.act16 = set()
            self.dyo = None

    def ymm_of(self, l) -> tuple:
        """(pointer, ld) of fused layer l's max keys; its min keys sit ld ints further."""
        half = self.ymm.numel() // 2
        return self.ymm.data_ptr() + 4 * self._ymm_idx[l.name] * self._ymm_C, half

    def _wire_fused_bn_bwd(self, eng, L, kinds):
        """Fused layers read g and write their dgrad without a dy buffer in between, so g and the dgrad output
        must differ: walking the backward order, each fused layer writes its dgrad into the other buffer of its
        resolution's pair (G, D), which becomes the g of the layer before it.  Non-fused layers keep dy in D
        (in place when their g already sits in D: the mode-0 apply is elementwise, index for index)."""
        self.fused = {l.name for l in L if eng.fuses_bn_bwd(l, kinds[l.name], self.B)}
        self.g_amax_key = {}
        self.out0_g_key = None
        if not self.fused:
            return
        other = {}
        for a_, b_ in ((self.G0, self.D0), (self.G1, self.D1)):
            other[a_.data_ptr()], other[b_.data_ptr()] = b_, a_
        idx = {l.name: i for i, l in enumerate(L)}
        for l in reversed(L):
            if l.name not in self.fused:
                continue
            if idx[l.name] + 1 < len(L):
                nxt = L[idx[l.name] + 1]                  # its g is written (last) by the next layer's dgrad
                self.g_amax_key[nxt.name] = "g:" + l.name
            else:                                         # up2's last conv ("plain"): g is out.0's dgrad output
                self.out0_g_key = "g:" + l.name
            g = self.gout[l.name]
            if l.name in ("down1.model.0.conv1", "down2.model.0.conv1"):
                continue                                  # dgrad accumulates into a concat-grad slice
            # g of a "plain" / "resid" layer is a slice of the concat gradient: any buffer of the pair is free
            dst = other.get(g.buf.data_ptr(), self.G0 if l.S == self.eng.H else self.G1)
            self.dgrad_dst[l.name] = Act(dst, l.cin)
            if l.name == "up1.model.1.conv1":
                self.gT1 = dst
            elif l.name == "up2.model.1.conv1":
                self.gT2 = dst
            else:
                prev = L[idx[l.name] - 1]
                assert kinds[prev.name] == "dense", prev.name
                self.gout[prev.name] = Act(dst, prev.cout)

    def _slab_floats(self):
        eng, B = self.eng, self.B
        nf, H = eng.nf, eng.H
        P0 = B * H * H
        need = _cdiv(P0, CHUNK) * 10 * 2 * nf          # stats / bwd partials at full res (R <= 10)
        need = max(need, B * H // cout1_band_rows(B, H) * 9 * nf)   # out.3 weight-gradient band partials
        if self.train:
            for l in eng.layers:                         # conv wgrad split-K slabs
                if l.cin > 1:
                    sp = wgrad_splits(B * l.S * l.S, l.cout, 9 * l.cin)
                    need = max(need, sp * l.cout * 9 * l.cin)
            # out.0 (2nf -> nf at full resolution; not in eng.layers)
            need = max(need, wgrad_splits(P0, nf, 9 * 2 * nf) * nf * 9 * 2 * nf)
            if eng.cp > 1:                                  # out.3 (nf -> in_channels) on the general weight gradient
                need = max(need, wgrad_splits(P0, eng.cp, 9 * nf) * eng.cp * 9 * nf)
            for cin, Hin in ((4 * nf, H // 4), (2 * nf, H // 2)):   # convT wgrad
                need = max(need, wgrad_splits(B * Hin * Hin, cin, 4 * nf) * cin * 4 * nf)
            if not (eng.up0_large and B <= 16):             # up0 weight grad through a split-K slab
                need = max(need, 2 * nf * eng.KK0 * 2 * nf)
            need = max(need, 64 * B * 2 * nf)               # up0 dgrad split-K
            if eng.up0_large:                               # cdm_up0_dgrad partials (32768-wide K ranges)
                need = max(need, _cdiv(2 * nf * eng.KK0, 32768) * B * 2 * nf)
        return int(need)
