"""Where does the HIP eval forward lose accuracy on the T=1500 sampler states?  

Takes x_t states of the reference's fp64 trajectory (tests/golden/sampler_T1500_nf8.npz), runs ONE eval forward of
the nf=8 model on them with the HIP engine, the CPU oracle in fp32 (== the reference) and the oracle in fp64, and
prints per-intermediate errors vs fp64 (max|d| / max|ref64| and relative L2) for HIP and for the reference fp32 path.
Intermediates are read from the engine workspace (NHWC) after the forward.

    python tools/t1500_probe.py [--math h3] [--slots 25,50,74]
"""
import argparse
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import ref_cpu as R  # noqa: E402


def oracle_forward(sd, x, t, c, sc, nf, h=64):
    """unet_forward with its intermediates (ContextUnet.py:42-60)."""
    ctx = R._Ctx(sd, False)
    I = {}
    x0 = ctx.res_block(x, "init_conv", is_res=True, shortcut=sc); I["x0"] = x0
    d1 = ctx.down(x0, "down1"); I["d1"] = d1
    d2 = ctx.down(d1, "down2"); I["d2"] = d2
    hv = F.gelu(F.avg_pool2d(d2, h // 4)); I["hv"] = hv.reshape(hv.shape[0], -1)
    cemb1 = ctx.embed(c, "contextembed1", 6).view(-1, 2 * nf, 1, 1)
    temb1 = ctx.embed(t, "timeembed1", 1).view(-1, 2 * nf, 1, 1)
    cemb2 = ctx.embed(c, "contextembed2", 6).view(-1, nf, 1, 1)
    temb2 = ctx.embed(t, "timeembed2", 1).view(-1, nf, 1, 1)
    I["cemb1"], I["temb1"], I["cemb2"], I["temb2"] = (v.reshape(v.shape[0], -1) for v in (cemb1, temb1, cemb2, temb2))
    u1 = F.conv_transpose2d(hv, sd["up0.0.weight"], sd["up0.0.bias"], stride=h // 4); I["y0"] = u1
    u1 = F.relu(F.group_norm(u1, 8, sd["up0.1.weight"], sd["up0.1.bias"], eps=R.GN_EPS))
    f1 = cemb1 * u1 + temb1; I["film1"] = f1
    u2 = ctx.up(f1, d2, "up1")
    f2 = cemb2 * u2 + temb2; I["film2"] = f2
    u3 = ctx.up(f2, d1, "up2"); I["u3"] = u3
    o = torch.cat((u3, x0), 1)
    o = F.conv2d(o, sd["out.0.weight"], sd["out.0.bias"], padding=1); I["yO"] = o
    o = F.relu(F.group_norm(o, 8, sd["out.1.weight"], sd["out.1.bias"], eps=R.GN_EPS)); I["zO"] = o
    I["eps"] = F.conv2d(o, sd["out.3.weight"], sd["out.3.bias"], padding=1)
    return I


def nchw(a, B, S, C):
    return a.reshape(B, S, S, C).permute(0, 3, 1, 2).contiguous().cpu().double()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--math", default="h3")
    ap.add_argument("--slots", default="25,50,74,81")
    ap.add_argument("--w", type=float, default=0.0)
    a = ap.parse_args()
    import cdm_amd
    from cdm_amd.diffusion import snapshot_slots
    g = os.path.join(ROOT, "tests", "golden")
    fx = np.load(os.path.join(g, "model_nf8.npz"))
    sd = {k[3:]: torch.from_numpy(fx[k].copy()) for k in fx.files if k.startswith("sd.")}
    sfx = np.load(os.path.join(g, "sampler_T1500_nf8.npz"))
    T = int(sfx["T"]); nf = 8; H = 64
    params = torch.from_numpy(sfx["params"])
    slots, _ = snapshot_slots(T)
    keep = list(sfx["snap_keep"])
    m = cdm_amd.ContextUnet(1, nf, 6, H, conv_math=a.math)
    m.load_state_dict(sd)
    m = m.cuda().eval()
    eng, P = m._engine_and_params()
    s = torch.cuda.current_stream().cuda_stream
    eng.repack(P, False, s)
    B = 2
    ws = eng.workspace(B, False)
    sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}
    torch.manual_seed(0)
    scw, scb = R.draw_shortcut(1, nf)
    for slot in [int(v) for v in a.slots.split(",")]:
        j = keep.index(slot)
        i = int(np.nonzero(slots == slot)[0][0]) - 1      # the state after step slots==slot is x_{i}; next call i
        x64 = torch.from_numpy(sfx[f"w{a.w:g}_inter_fp64"][j]).double()
        x32 = x64.float()
        t = torch.tensor([i / T])
        I32 = oracle_forward(sd, x32, t, params, (scw, scb), nf)
        I64 = oracle_forward(sd64, x32.double(), t.double(), params.double(), (scw.double(), scb.double()), nf)
        xg = x32.cuda().reshape(B, H, H).contiguous()
        eps = eng.forward(ws, P, xg, t.cuda(), params.cuda().float(), scw.reshape(nf).cuda(), scb.cuda(), B, s)
        torch.cuda.synchronize()
        H1, H2 = H // 2, H // 4
        catO = nchw(ws.catO.buf, B, H, 2 * nf)
        catU2 = nchw(ws.catU2.buf, B, H1, 2 * nf)
        catU1 = nchw(ws.catU1.buf, B, H2, 4 * nf)
        hip = {"x0": catO[:, nf:], "u3": catO[:, :nf], "d1": catU2[:, nf:], "film2": catU2[:, :nf],
               "d2": catU1[:, 2 * nf:], "film1": catU1[:, :2 * nf], "hv": ws.hv.cpu().double(),
               "y0": nchw(ws.y0, B, H2, 2 * nf), "yO": nchw(ws.yO, B, H, nf),
               "eps": eps.reshape(B, 1, H, H).cpu().double()}
        for k in ("cemb1", "temb1", "cemb2", "temb2"):
            mname = {"cemb1": "contextembed1", "temb1": "timeembed1", "cemb2": "contextembed2",
                     "temb2": "timeembed2"}[k]
            hip[k] = ws.emb[mname].cpu().double()
        print(f"--- slot {slot} (step i={i}, max|x| {x64.abs().max():.4g}) [{a.math}]")
        print(f"{'tensor':8s} {'max|ref|':>10s} {'HIP max':>10s} {'ref32 max':>10s} {'HIP L2':>10s} {'ref32 L2':>10s}"
              f" {'ratio':>6s}")
        for k in ("x0", "d1", "d2", "hv", "cemb1", "temb1", "cemb2", "temb2", "y0", "film1", "film2", "u3", "yO",
                  "eps"):
            r = I64[k].double(); c_ = I32[k].double().reshape(r.shape)
            h_ = hip[k].reshape(-1)[: r.numel()].reshape(r.shape)   # broadcast t: one embedding row written
            mx = r.abs().max().item()
            l2 = r.norm().item()
            eh, ec = (h_ - r).abs().max().item() / mx, (c_ - r).abs().max().item() / mx
            lh, lc = (h_ - r).norm().item() / l2, (c_ - r).norm().item() / l2
            print(f"{k:8s} {mx:10.4g} {eh:10.3e} {ec:10.3e} {lh:10.3e} {lc:10.3e} {lh / max(lc, 1e-30):6.2f}")


if __name__ == "__main__":
    main()
