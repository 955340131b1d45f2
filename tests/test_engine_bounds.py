"""CPU dry run of the engine's launch sequence (no GPU): every library call of a train forward + backward is
recorded through a stand-in for the C-ABI library, then checked on the host — every pointer argument lies in a
live tensor of the run, and every split-K slab / fused-BN operand range fits its buffer.  Catches workspace
sizing and wiring errors before a kernel can fault on the GPU (the out.0 weight-gradient slab was once sized
only by the 18 BN layers: fine at B=256, an overflow at B=2, n_feat=128)."""
import ctypes
import os
import re

import pytest
import torch

import cdm_amd._lib as LL
import cdm_amd.engine as E

HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "cdm_hip.h")


def _param_names():
    src = re.sub(r"/\*.*?\*/", "", open(HDR).read(), flags=re.S)
    out = {}
    for m in re.finditer(r"\bint\s+(cdm_\w+)\s*\(([^;]*?)\)\s*;", src, flags=re.S):
        out[m.group(1)] = [p.strip().split()[-1].lstrip("*") for p in m.group(2).split(",") if p.strip()]
    return out


def _eff_splits(K, s, bk=16):
    kt = (K + bk - 1) // bk
    s = max(1, min(s, kt))
    per = (kt + s - 1) // s
    return (kt + per - 1) // per if kt > 0 else 1


class _Recorder:
    def __init__(self, protos):
        self.protos, self.calls = protos, []

    def __getattr__(self, name):
        if name in self.protos:
            return lambda *a: self.calls.append((name, a)) or 0
        if name == "raw":
            return lambda n: (lambda K, s: _eff_splits(K, s)) if n == "cdm_gemm_splits" else (lambda *a: 0)
        raise AttributeError(name)


def _dry_run(monkeypatch, nf, B, math, H=64, train=True):
    protos = LL.parse_header()
    rec = _Recorder(protos)
    monkeypatch.setattr(E, "lib", lambda: rec)
    eng = E.UNetEngine(nf, 6, H, "cpu", math)
    _dry_run.last_eng = eng
    from cdm_amd.model import ContextUnet
    torch.manual_seed(0)
    m = ContextUnet(1, nf, 6, H, conv_math=math)
    P = {k: v.detach().clone() for k, v in list(m.named_parameters()) + list(m.named_buffers())}
    eng.repack(P, train, 0)
    ws = eng.workspace(B, train)
    x, t, c = torch.empty(B, H, H), torch.rand(B), torch.rand(B, 6)
    sc_w, sc_b = torch.rand(2 * nf), torch.rand(2 * nf)
    eng.forward(ws, P, x, t if train else t[:1], c, sc_w, sc_b, B if train else B // 2, 0)
    G = {n: torch.empty_like(v) for n, v in m.named_parameters()}
    deps = torch.empty(B, H, H)
    if train:
        eng.backward(ws, P, deps, G, 0)
    live = []

    def reg(o):
        if isinstance(o, torch.Tensor) and o.numel():
            live.append((o.data_ptr(), o.data_ptr() + o.numel() * o.element_size()))
        elif isinstance(o, E.Act):
            reg(o.buf)
        elif isinstance(o, dict):
            for v in o.values():
                reg(v)
        elif isinstance(o, (list, tuple)):
            for v in o:
                reg(v)
    for o in (P, G, eng.pk, vars(ws), [x, t, c, sc_w, sc_b, deps, eng._amax, eng._ones, eng._zeros],
              [getattr(eng, "_batch_jobs", None), getattr(eng, "_batch_slots", None)]):
        reg(o)
    return rec.calls, protos, live


def _region(live, p):
    for a, b in live:
        if a <= p < b:
            return a, b
    return None


# The bench shapes run at full size: the workspaces are torch.empty on the host, which the kernel commits only when
# touched, so B=256 (~20 GB of address space) costs < 1 GB of RSS.  Train: C2 (n_feat=128, B=256), C5 (n_feat=256,
# 256x256, B=16); eval (sampler): the CFG batch of C2 (2 x 256 images, cond + uncond halves).
@pytest.mark.parametrize("nf,B,math,H,train", [(128, 2, "h3", 64, True), (128, 3, "fp32", 64, True),
                                               (64, 2, "h3", 64, True), (16, 1, "x6", 64, True),
                                               (128, 256, "h3", 64, True), (128, 256, "bf16", 64, True),
                                               (128, 1, "h3", 256, True), (256, 16, "h3", 256, True),
                                               (16, 20, "h3", 256, True),
                                               (128, 512, "h3", 64, False), (256, 32, "h3", 256, False)])
def test_launch_arguments_stay_in_bounds(monkeypatch, nf, B, math, H, train):
    calls, protos, live = _dry_run(monkeypatch, nf, B, math, H, train)
    names = _param_names()
    assert len(calls) > (100 if train else 40)
    problems = []

    def need(name, a, ptr, nbytes, what):
        r = _region(live, ptr)
        if r is None:
            problems.append(f"{name}: {what} not in a live tensor")
        elif ptr + nbytes > r[1]:
            problems.append(f"{name}: {what} overruns its buffer by {ptr + nbytes - r[1]} bytes")

    for name, args in calls:
        pn = names[name]
        a = dict(zip(pn, args))
        for (pname, v), ty in zip(zip(pn, args), protos[name]):
            if ty is ctypes.c_void_p and isinstance(v, int) and v and name not in ("cdm_embed_fwd", "cdm_embed_bwd"):
                if _region(live, v) is None:
                    problems.append(f"{name}: pointer {pname} not in a live tensor")
        if name.startswith("cdm_conv3x3_wgrad"):
            K = a["N"] * a["H"] * a["W"]
            need(name, a, a["slab"], _eff_splits(K, a["splits"]) * a["Cout"] * 9 * a["Cin"] * 4, "slab")
        elif name.startswith("cdm_convT2x2_wgrad"):
            K = a["N"] * a["H"] * a["W"]
            need(name, a, a["slab"], _eff_splits(K, a["splits"]) * a["Cin"] * 4 * a["Cout"] * 4, "slab")
        elif name == "cdm_gemm_tn_f32":
            need(name, a, a["slab"], _eff_splits(a["K"], a["splits"]) * a["M"] * a["N"] * 4, "slab")
        elif name == "cdm_gemm_f32" and _eff_splits(a["K"], a["splits"]) > 1:
            need(name, a, a["slab"], _eff_splits(a["K"], a["splits"]) * a["M"] * a["N"] * 4, "slab")
        elif name == "cdm_conv3x3_cout1_wgrad":
            nblk = a["N"] * a["H"] // -a["csize"] if a["csize"] < 0 else a["N"] * -(-a["H"] * a["W"] // a["csize"])
            need(name, a, a["slab"], nblk * 9 * a["C"] * 4, "slab")
        elif name == "cdm_slab_reduce":
            need(name, a, a["slab"], a["splits"] * a["M"] * a["N"] * 4, "slab")
        if name == "cdm_pack_split_conv3x3_batch":
            import numpy as np
            tab = _dry_run.last_eng._batch_jobs.numpy()
            assert a["jobs_dev"] == _dry_run.last_eng._batch_jobs.data_ptr() and a["njobs"] * 48 == tab.size
            for j in range(a["njobs"]):
                rec = tab[48 * j:48 * (j + 1)]
                Wp, wx, wd, am = (int(np.frombuffer(rec[o:o + 8].tobytes(), np.uint64)[0]) for o in (0, 24, 32, 40))
                cin, cout, kc = (int(np.frombuffer(rec[o:o + 4].tobytes(), np.int32)[0]) for o in (8, 12, 16))
                assert cin * cout * 9 <= a["max_w_elems"]
                need(name, a, Wp, cin * cout * 9 * 4, f"job {j} W")
                need(name, a, wx, -(-9 * cin // 16) * 3 * cout * 16 * 2, f"job {j} wpk_x")
                if wd:
                    need(name, a, wd, -(-9 * cout // 16) * 3 * cin * 16 * 2, f"job {j} wdg_x")
                need(name, a, am, 4, f"job {j} amax")
        if name == "cdm_conv3x3_fwd_h3_ex":
            Pn = a["N"] * a["H"] * a["W"]
            need(name, a, a["x"], ((Pn - 1) * a["ldx"] + a["Cin"]) * 4, "x")
            need(name, a, a["y"], ((Pn - 1) * a["ldy"] + a["Cout"]) * 4, "y")
            if a["pre_s"]:
                need(name, a, a["pre_s"], a["Cin"] * 4, "pre_s"); need(name, a, a["pre_t"], a["Cin"] * 4, "pre_t")
            if a["ymm"]:
                need(name, a, a["ymm"], a["Cout"] * 4, "ymm max")
                need(name, a, a["ymm"] + 4 * a["ymm_ld"], a["Cout"] * 4, "ymm min")
        if name == "cdm_conv3x3_wgrad_h3_ex":
            Pn = a["N"] * a["H"] * a["W"]
            need(name, a, a["g"], ((Pn - 1) * a["ldg"] + a["Cout"]) * 4, "g")
            if a["y"]:
                need(name, a, a["y"], ((Pn - 1) * a["ldy"] + a["Cout"]) * 4, "y")
            need(name, a, a["x"], ((Pn - 1) * a["ldx"] + a["Cin"]) * 4, "x")
            if a["x_s"]:
                need(name, a, a["x_s"], a["Cin"] * 4, "x_s"); need(name, a, a["x_t"], a["Cin"] * 4, "x_t")
            K = a["N"] * a["H"] * a["W"]
            need(name, a, a["slab"], _eff_splits(K, a["splits"]) * a["Cout"] * 9 * a["Cin"] * 4, "slab")
        if name == "cdm_bn_fwd_finalize" and a["ymm"]:
            need(name, a, a["ymm"], a["C"] * 4, "ymm max")
            need(name, a, a["ymm"] + 4 * a["ymm_ld"], a["C"] * 4, "ymm min")
        if name == "cdm_conv3x3_dgrad_h3_bnbwd":
            Pn = a["N"] * a["H"] * a["W"]
            need(name, a, a["g"], ((Pn - 1) * a["ldg"] + a["C"]) * 4, "g")
            need(name, a, a["y"], ((Pn - 1) * a["ldy"] + a["C"]) * 4, "y")
            need(name, a, a["out"], ((Pn - 1) * a["ldo"] + a["Cout"]) * 4, "out")
        if name == "cdm_conv3x3_wgrad_h3_bnbwd":
            Pn = a["N"] * a["H"] * a["W"]
            need(name, a, a["g"], ((Pn - 1) * a["ldg"] + a["Cout"]) * 4, "g")
            need(name, a, a["y"], ((Pn - 1) * a["ldy"] + a["Cout"]) * 4, "y")
            need(name, a, a["x"], ((Pn - 1) * a["ldx"] + a["Cin"]) * 4, "x")
    assert not problems, problems[:10]
