"""Per-step local errors along the T=1500 nf=8 trajectory.

Runs the reference sampler loop (code/train_diffusion_condition.py:312-333, CPU-RNG order: x_T, then per step z and the
fresh shortcut) with the HIP eval forward, and at every step also evaluates the CPU oracle in fp32 (== the reference)
and in fp64 on the same state x_t, t, c and shortcut.  Prints, per window of steps, the eps error vs fp64 of HIP and of
the reference fp32 path: the per-step max / L2, and the L2 of the error summed over the window (a coherent error —
the same sign at a pixel step after step — grows linearly in that sum, a random one like sqrt(steps)).

    python tools/t1500_steps.py [--w 0] [--math h3] [--window 100]
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import ref_cpu as R  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from t1500_probe import nchw, oracle_forward  # noqa: E402

KEYS = ("x0", "d1", "d2", "hv", "cemb1", "temb1", "cemb2", "temb2", "y0", "film1", "film2", "u3", "yO", "eps")


def hip_intermediates(ws, eps, B, H, nf):
    H1, H2 = H // 2, H // 4
    catO = nchw(ws.catO.buf, B, H, 2 * nf)
    catU2 = nchw(ws.catU2.buf, B, H1, 2 * nf)
    catU1 = nchw(ws.catU1.buf, B, H2, 4 * nf)
    out = {"x0": catO[:, nf:], "u3": catO[:, :nf], "d1": catU2[:, nf:], "film2": catU2[:, :nf],
           "d2": catU1[:, 2 * nf:], "film1": catU1[:, :2 * nf], "hv": ws.hv.cpu().double(),
           "y0": nchw(ws.y0, B, H2, 2 * nf), "yO": nchw(ws.yO, B, H, nf), "eps": eps.reshape(B, 1, H, H).cpu().double()}
    for k, mname in (("cemb1", "contextembed1"), ("temb1", "timeembed1"), ("cemb2", "contextembed2"),
                     ("temb2", "timeembed2")):
        out[k] = ws.emb[mname].cpu().double()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--w", type=float, default=0.0)
    ap.add_argument("--math", default="h3")
    ap.add_argument("--window", type=int, default=100)
    ap.add_argument("--steps", type=int, default=1500)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--layers", action="store_true", help="per-intermediate cumulative errors (w = 0)")
    ap.add_argument("--override", default="", help="comma list of x0,d1,d2,emb,film2,u3,yO,eps: substitute the fp64 oracle's "
                                                     "value (rounded to fp32) there in every HIP forward (w = 0)")
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    import cdm_amd
    g = os.path.join(ROOT, "tests", "golden")
    fx = np.load(os.path.join(g, "model_nf8.npz"))
    sd = {k[3:]: torch.from_numpy(fx[k].copy()) for k in fx.files if k.startswith("sd.")}
    sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}
    sfx = np.load(os.path.join(g, "sampler_T1500_nf8.npz"))
    T = int(sfx["T"]); nf, H, n = 8, 64, 2
    params = torch.from_numpy(sfx["params"])
    m = cdm_amd.ContextUnet(1, nf, 6, H, conv_math=a.math)
    m.load_state_dict(sd)
    m = m.cuda().eval()
    eng, P = m._engine_and_params()
    s = torch.cuda.current_stream().cuda_stream
    eng.repack(P, False, s)
    cfg = a.w > 0
    B = 2 * n if cfg else n
    ws = eng.workspace(B, False)
    sched = cdm_amd.Schedule(T, "cuda")
    b32, a32, ab32 = R.make_schedule(T)
    torch.manual_seed(int(sfx[f"w{a.w:g}_seed"]))
    x = torch.randn(n, 1, H, H)
    cpar = torch.cat([params, torch.zeros_like(params)]) if cfg else params
    xh = x.cuda()
    acc_h = torch.zeros(n, 1, H, H, dtype=torch.float64); acc_r = torch.zeros_like(acc_h)
    rows = []
    lay_h, lay_r, lay_n = {}, {}, {}
    overrides = {v for v in a.override.split(",") if v}
    assert not (overrides and cfg)
    t0 = time.time()
    for k, i in enumerate(range(T, T - a.steps, -1)):
        z = torch.randn(n, 1, H, H) if i > 1 else None
        scs = [R.draw_shortcut(1, nf) for _ in range(2 if cfg else 1)]
        t = torch.tensor([i / T])
        xs = xh.cpu()
        xin = torch.cat([xs, xs]) if cfg else xs
        scw = torch.cat([w.reshape(nf) for w, _ in scs]); scb = torch.cat([b for _, b in scs])
        if overrides:
            I64o = oracle_forward(sd64, xs.double(), t.double(), params.double(),
                                  (scs[0][0].double(), scs[0][1].double()), nf)

            def nhwc(v):
                return v.float().permute(0, 2, 3, 1).contiguous().cuda()

            def stage(name, ws_):
                if name not in overrides:
                    return
                H1, H2 = H // 2, H // 4
                if name == "x0":
                    ws_.catO.buf.view(n, H, H, 2 * nf)[..., nf:] = nhwc(I64o["x0"])
                elif name == "u3":
                    ws_.catO.buf.view(n, H, H, 2 * nf)[..., :nf] = nhwc(I64o["u3"])
                elif name == "d1":
                    ws_.catU2.buf.view(n, H1, H1, 2 * nf)[..., nf:] = nhwc(I64o["d1"])
                elif name == "film2":
                    ws_.catU2.buf.view(n, H1, H1, 2 * nf)[..., :nf] = nhwc(I64o["film2"])
                elif name == "d2":
                    ws_.catU1.buf.view(n, H2, H2, 4 * nf)[..., 2 * nf:] = nhwc(I64o["d2"])
                elif name == "yO":      # out.0's pre-norm output; its GroupNorm statistics come from the conv epilogue
                    ws_.yO.view(n, H, H, nf)[:] = nhwc(I64o["yO"])
                    ws_.slab.zero_()
                    yo = I64o["yO"].double()                      # exact per-(image, 128-pixel chunk) sums
                    v = yo.permute(0, 2, 3, 1).reshape(n, H * H // 128, 128, nf)
                    sl = torch.stack([v.sum(2), (v * v).sum(2)], 2).float().reshape(-1)
                    ws_.slab[: sl.numel()] = sl.cuda()
                elif name == "emb":
                    for k_, mname in (("cemb1", "contextembed1"), ("temb1", "timeembed1"), ("cemb2", "contextembed2"),
                                      ("temb2", "timeembed2")):
                        v = I64o[k_].float().cuda()
                        ws_.emb[mname][: v.shape[0]] = v
            eng.stage_probe = stage
        e = eng.forward(ws, P, xin.cuda().reshape(B, H, H).contiguous(), t.cuda(), cpar.cuda(), scw.cuda(),
                        scb.cuda(), n, s).reshape(B, 1, H, H).clone()

        def orc(sdx, dt):
            outs = []
            for j, (w_, b_) in enumerate(scs):
                cc = params if j == 0 else torch.zeros_like(params)
                with torch.no_grad():
                    outs.append(R.unet_forward(sdx, xs.to(dt), t.to(dt), cc.to(dt), n_feat=nf, n_cfeat=6, height=H,
                                               train=False, shortcut=(w_.to(dt), b_.to(dt))))
            return outs

        o32, o64 = orc(sd, torch.float32), orc(sd64, torch.float64)
        if a.layers and not cfg:                 # per-intermediate errors (w = 0: one forward per step)
            I32 = oracle_forward(sd, xs, t, params, scs[0], nf)
            I64 = oracle_forward(sd64, xs.double(), t.double(), params.double(),
                                 (scs[0][0].double(), scs[0][1].double()), nf)
            HI = hip_intermediates(ws, e, n, H, nf)
            for key in KEYS:
                r = I64[key].double()
                h_ = HI[key].reshape(-1)[: r.numel()].reshape(r.shape)
                lay_h[key] = lay_h.get(key, 0) + (h_ - r)
                lay_r[key] = lay_r.get(key, 0) + (I32[key].double().reshape(r.shape) - r)
                lay_n[key] = lay_n.get(key, 0.0) + r.norm().item()
        if "eps" in overrides:
            e = I64o["eps"].float().cuda().reshape(B, 1, H, H)
        if cfg:
            eh = e[n:] + a.w * (e[:n] - e[n:])
            e32 = o32[1] + a.w * (o32[0] - o32[1])
            e64 = o64[1] + a.w * (o64[0] - o64[1])
        else:
            eh, e32, e64 = e, o32[0], o64[0]
        dh = eh.cpu().double() - e64; dr = e32.double() - e64
        acc_h += dh; acc_r += dr
        rows.append((i, dh.abs().max().item(), dr.abs().max().item(), dh.norm().item(), dr.norm().item(),
                     e64.norm().item()))
        xh = cdm_amd.denoise_add_noise(xh, i, eh.cuda() if not eh.is_cuda else eh, z.cuda() if z is not None else 0,
                                       sched)
        if (k + 1) % a.window == 0 or i == T - a.steps + 1:
            blk = rows[-a.window:]
            mh = np.mean([r[3] for r in blk]); mr = np.mean([r[4] for r in blk]); ne = np.mean([r[5] for r in blk])
            print(f"steps {blk[0][0]:5d}..{blk[-1][0]:5d}: per-step L2 err / |eps|  HIP {mh / ne:.3e}  ref32 {mr / ne:.3e}"
                  f"  | cumulative-sum L2  HIP {acc_h.norm().item():.3e}  ref32 {acc_r.norm().item():.3e}"
                  f"  | max|x| {xh.abs().max().item():.4g}  ({time.time() - t0:.0f} s)", flush=True)
            if lay_h:
                print("    cumulative-sum L2 / sum of |ref|, HIP vs ref32: " + ", ".join(
                    f"{key} {lay_h[key].norm().item() / lay_n[key]:.2e}/{lay_r[key].norm().item() / lay_n[key]:.2e}"
                    for key in KEYS), flush=True)
    ref64 = sfx[f"w{a.w:g}_x_fp64"]
    if a.steps == T:
        mx = np.abs(ref64).max()
        print(f"final x vs fp64: HIP (this loop) {np.abs(xh.cpu().numpy() - ref64).max() / mx:.3e}, reference fp32 "
              f"{np.abs(sfx[f'w{a.w:g}_x'] - ref64).max() / mx:.3e}")
        dh = xh.cpu().numpy() - ref64
        dr = sfx[f"w{a.w:g}_x"] - ref64
        for name, d in (("HIP", dh), ("ref32", dr)):
            k = np.unravel_index(np.abs(d).argmax(), d.shape)
            print(f"  {name}: argmax {tuple(int(v) for v in k)} d {d[k]:.4g} x64 {ref64[k]:.6g} | L2 rel "
                  f"{np.linalg.norm(d) / np.linalg.norm(ref64):.3e} | corr(HIP, ref32) "
                  f"{float((dh * dr).sum() / np.linalg.norm(dh) / np.linalg.norm(dr)):.3f}")
        np.savez_compressed(os.path.join(ROOT, "gpurun_out", f"t1500_final_{a.override or 'none'}.npz"),
                            x_hip=xh.cpu().numpy(), x64=ref64, x32=sfx[f"w{a.w:g}_x"])


if __name__ == "__main__":
    main()
