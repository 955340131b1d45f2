"""Kink audit of the input-gradient test inputs (VERDICT r4 "next" 2): per normalisation layer of ContextUnet
(n_feat = 16, B = 4, train-mode BatchNorm), HIP's pre-activations z = y s + t vs the CPU oracle in fp32 (the reference's
arithmetic) and fp64: relative error of y, of the batch mean / invstd, and the ReLU / MaxPool decisions that differ from
fp64 (count and the |z64| of the flipped elements).

    python tools/kink_diag.py [seeds] [math]        e.g.  python tools/kink_diag.py 0,1,8 fp32

Test infrastructure (imports oracle/), never on the product path.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from oracle import ref_cpu as R  # noqa: E402

NF, NCF, H, B = 16, 6, 64, 4


def _inputs(seed, math):
    import cdm_amd
    torch.manual_seed(3 + 100 * seed)
    m = cdm_amd.ContextUnet(1, NF, NCF, H, conv_math=math).cuda().train()
    sd = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    g = torch.Generator().manual_seed(11 + 100 * seed)
    x = torch.randn(B, 1, H, H, generator=g)
    t = torch.rand(B, generator=g)
    c = torch.rand(B, NCF, generator=g)
    torch.manual_seed(21)
    sc = R.draw_shortcut(1, NF)
    return m, sd, x, t, c, sc


def _oracle_layers(sd, x, t, c, sc, dtype):
    """{layer: (y NHWC [npix, C] float64, zpre NHWC float64, mean, invstd)} of the oracle forward in `dtype`."""
    sd = {k: (v.to(dtype) if v.is_floating_point() else v.clone()).clone() for k, v in sd.items()}
    out = {}
    orig_bn = R._Ctx.bn
    orig_gn = F.group_norm

    def bn(self, y, name):
        z = orig_bn(self, y, name)
        mean = y.mean(dim=(0, 2, 3)); var = y.var(dim=(0, 2, 3), unbiased=False)
        out[name[:-2]] = (y, z, mean, (var + 1e-5).rsqrt())
        return z

    def gn(y, G, w, b, eps=1e-5):
        z = orig_gn(y, G, w, b, eps=eps)
        out["up0" if "up0" not in out else "out.0"] = (y, z, None, None)
        return z
    R._Ctx.bn = bn
    F.group_norm = gn
    try:
        with torch.no_grad():
            eps = R.unet_forward(sd, x.to(dtype), t.to(dtype), c.to(dtype), n_feat=NF, n_cfeat=NCF, height=H, train=True,
                                 shortcut=(sc[0].to(dtype), sc[1].to(dtype)))
    finally:
        R._Ctx.bn = orig_bn
        F.group_norm = orig_gn
    nhwc = lambda v: v.permute(0, 2, 3, 1).reshape(-1, v.shape[1]).double().numpy()   # noqa: E731
    return {k: (nhwc(y), nhwc(z), None if m is None else m.double().numpy(), None if s is None else s.double().numpy())
            for k, (y, z, m, s) in out.items()}, eps.double().numpy()


def _hip_layers(m, x, t, c, sc):
    eng, P = m._engine_and_params()
    s = torch.cuda.current_stream().cuda_stream
    eng.repack(P, True, s)
    ws = eng.workspace(B, True)
    eps = eng.forward(ws, P, x.cuda().reshape(B, H, H), t.cuda(), c.cuda(), sc[0].reshape(-1).cuda(), sc[1].cuda(), B, s)
    torch.cuda.synchronize()
    out = {}
    for l in eng.layers:
        y = ws.y[l.name].float().cpu().double().numpy().reshape(-1, l.cout)
        st = {k: v.cpu().double().numpy() for k, v in ws.bn[l.name].items()}
        z = (y * st["scale"] + st["shift"]).astype(np.float32).astype(np.float64)
        out[l.name] = (y, z, st["mean"], st["invstd"])
    for key, yb, st, C in (("up0", ws.y0, ws.gn0, 2 * NF), ("out.0", ws.yO, ws.gnO, NF)):
        y = yb.cpu().double().numpy().reshape(B, -1, C)
        sc_ = st["scale"].cpu().double().numpy().reshape(B, 1, C); sh = st["shift"].cpu().double().numpy().reshape(B, 1, C)
        out[key] = (y.reshape(-1, C), (y * sc_ + sh).astype(np.float32).astype(np.float64).reshape(-1, C), None, None)
    return out, eps.cpu().double().numpy().reshape(B, 1, H, H)


def _rel(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def _pool_flips(z, z64, S, C):
    """MaxPool2d(2) argmax decisions (on relu(z)) that differ from fp64's."""
    def arg(zz):
        r = np.maximum(zz.reshape(B, S // 2, 2, S // 2, 2, C), 0).transpose(0, 1, 3, 5, 2, 4).reshape(-1, 4)
        return r.argmax(1), np.sort(r, 1)
    a, _ = arg(z)
    a64, s64 = arg(z64)
    flip = a != a64
    gap = (s64[:, 3] - s64[:, 2])[flip]
    return int(flip.sum()), (float(gap.min()) if flip.any() else None)


def audit(seed, math):
    m, sd, x, t, c, sc = _inputs(seed, math)
    o32, e32 = _oracle_layers(sd, x, t, c, sc, torch.float32)
    o64, e64 = _oracle_layers(sd, x, t, c, sc, torch.float64)
    hip, eh = _hip_layers(m, x, t, c, sc)
    rows = []
    pools = {"down1.model.1.conv2": 64, "down2.model.1.conv2": 32}
    for name in list(hip):
        if name not in o64:
            continue
        y64, z64, m64, s64 = o64[name]
        row = {"layer": name}
        for tag, src in (("hip", hip), ("ref32", o32)):
            y, z, mu, istd = src[name]
            row[f"y_err_{tag}"] = _rel(y, y64)
            if mu is not None and m64 is not None:
                row[f"mean_err_{tag}"] = float(np.abs(mu - m64).max() / np.abs(m64).max())
                row[f"invstd_err_{tag}"] = float(np.abs(istd / s64 - 1).max())
            # decisions near the kink: relu(z) positive in one, non-positive in the other
            fl = (z > 0) != (z64 > 0)
            row[f"relu_flips_{tag}"] = int(fl.sum())
            if fl.any():
                row[f"relu_flip_min_abs_z64_{tag}"] = float(np.abs(z64[fl]).max())
                row[f"relu_flip_abs_dz_{tag}"] = float(np.abs(z - z64)[fl].max())
            row[f"z_err_{tag}"] = float(np.abs(z - z64).max() / np.abs(z64).max())
            if name in pools:
                row[f"pool_flips_{tag}"], row[f"pool_flip_gap64_{tag}"] = _pool_flips(z, z64, pools[name], z.shape[1])
        rows.append(row)
    return {"seed": seed, "math": math, "eps_err_hip": _rel(eh, e64), "eps_err_ref32": _rel(e32, e64), "layers": rows}


if __name__ == "__main__":
    torch.set_num_threads(min(16, len(os.sched_getaffinity(0))))
    seeds = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "0,1,2").split(",")]
    maths = (sys.argv[2] if len(sys.argv) > 2 else "fp32,h3").split(",")
    for sd_ in seeds:
        for mth in maths:
            r = audit(sd_, mth)
            print(json.dumps(r), flush=True)
