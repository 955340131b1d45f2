"""Diagnostic (GPU box): the eval-mode BatchNorm weight gradient of up2.model.2.conv2 in
tests/test_gpu_input_grads.py::test_eval_mode_grads_vs_autograd[h3-0].

Runs the test's model / inputs on cuda:0 under each arithmetic, keeps the engine workspace of the autograd call and
saves what the layer's gradient is made of: the layer's pre-norm output y, the gradient g arriving at its ReLU output
(the first n_feat channels of the catO gradient buffer), the running statistics, and HIP's gamma / beta gradients.
The CPU side (tools/eval_dgamma_diag.py --analyse) compares them with fp64 autograd of the oracle on HIP's branch.

    python tools/eval_dgamma_diag.py gpurun_out/eval_dgamma.npz            # on the box
    python tools/eval_dgamma_diag.py --analyse gpurun_out/eval_dgamma.npz  # here
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

NF, NCF, H, B = 16, 6, 64, 4
LAYER = "up2.model.2.conv2"


def inputs(seed):
    g = torch.Generator().manual_seed(11 + 100 * seed)
    warm = [(torch.randn(B, 1, H, H, generator=g), torch.rand(B, generator=g), torch.rand(B, NCF, generator=g))
            for _ in range(2)]
    x = torch.randn(B, 1, H, H, generator=g)
    t = torch.rand(B, generator=g)
    c = torch.rand(B, NCF, generator=g)
    weight = torch.randn(B, 1, H, H, generator=g)
    return warm, x, t, c, weight


def run_box(out):
    import cdm_amd
    from cdm_amd import engine as E
    res = {}
    for math in ("fp32", "h3"):
        warm, x, t, c, weight = inputs(0)
        torch.manual_seed(3)                     # the test's construction order (seeded init, then the warm forwards)
        m = cdm_amd.ContextUnet(1, NF, NCF, H, conv_math=math).cuda().train()
        with torch.no_grad():
            for xx, tt, cc in warm:
                m(xx.cuda(), tt.cuda(), cc.cuda())
        m.eval()
        sd = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
        kept = {}
        orig = E.UNetEngine.backward
        orig_gn = E.UNetEngine._gn_bwd

        def gn_bwd(self, ws, P, name, *a, **kw):   # dyO = dL/d out.0's output, right after out.1's GroupNorm backward
            r = orig_gn(self, ws, P, name, *a, **kw)
            if name == "out.1":
                torch.cuda.synchronize()
                kept["dyO"] = ws.D0.view(-1)[: ws.B * H * H * NF].detach().cpu().clone()
            return r
        E.UNetEngine._gn_bwd = gn_bwd

        def bwd(self, ws, *a, **kw):
            r = orig(self, ws, *a, **kw)
            torch.cuda.synchronize()
            kept["y"] = ws.y[LAYER].detach().cpu().clone()
            kept["g"] = ws.dcatO.buf.detach().cpu().clone()
            return r
        E.UNetEngine.backward = bwd
        try:
            xg, tg, cg = (v.cuda().requires_grad_(True) for v in (x, t, c))
            torch.manual_seed(21)
            eps = m(xg, tg, cg)
            (eps * weight.cuda()).sum().backward()
        finally:
            E.UNetEngine.backward = orig
            E.UNetEngine._gn_bwd = orig_gn
        res[math + "_dyO"] = kept["dyO"].numpy()
        gr = {k: p.grad.detach().cpu() for k, p in m.named_parameters()}
        res[math + "_y"] = kept["y"].numpy()
        res[math + "_g"] = kept["g"].numpy()
        res[math + "_dgamma"] = gr[LAYER + ".1.weight"].numpy()
        res[math + "_dbeta"] = gr[LAYER + ".1.bias"].numpy()
        for k, v in sd.items():
            res[math + "_sd_" + k] = v.numpy()
    np.savez(out, **res)
    print("saved", out)


def analyse(path):
    from oracle import ref_cpu as R
    from _kinks import Kinks, hip_kinks  # noqa: F401
    import torch.nn.functional as F
    d = np.load(path)
    _, x, t, c, weight = inputs(0)
    torch.manual_seed(21)
    sc = R.draw_shortcut(1, NF)
    for math in ("fp32", "h3"):
        sd = {k[len(math) + 4:]: torch.from_numpy(d[k]) for k in d.files if k.startswith(math + "_sd_")}
        # fp64 on the fp32 oracle's branch (the HIP branch differs by no decision in the recorded runs: 0 flips)
        rec = {}
        orig = F.batch_norm

        def bn(inp, rm, rv, w=None, b=None, training=False, momentum=0.1, eps=1e-5):
            out = orig(inp, rm, rv, w, b, training, momentum, eps)
            k = len(rec)
            rec[k] = {"x": inp.detach().clone()}
            if out.requires_grad:
                out.register_hook(lambda gr_, k=k: rec[k].__setitem__("gbn", gr_.detach().clone()))
            return out
        conv_rec = {}
        orig_conv = F.conv2d

        def conv(inp, w, b=None, stride=1, padding=0, *a):
            out = orig_conv(inp, w, b, stride, padding, *a)
            if tuple(w.shape) == (NF, 2 * NF, 3, 3) and out.requires_grad:     # out.0
                conv_rec["w"] = w.detach().clone()
                out.register_hook(lambda gr_: conv_rec.__setitem__("dyO", gr_.detach().clone()))
            return out

        def run(dtype, kinks):
            rec.clear()
            R.F.conv2d = conv
            s = {k: (v.to(dtype) if v.is_floating_point() else v.clone()).clone() for k, v in sd.items()}
            for k, v in s.items():
                if v.is_floating_point() and "running" not in k:
                    v.requires_grad_(True)
            R.F.batch_norm = bn
            try:
                with kinks:
                    e = R.unet_forward(s, x.to(dtype), t.to(dtype), c.to(dtype), n_feat=NF, n_cfeat=NCF, height=H,
                                       train=False, shortcut=(sc[0].to(dtype), sc[1].to(dtype)))
                (e * weight.to(dtype)).sum().backward()
            finally:
                R.F.batch_norm = orig
                R.F.conv2d = orig_conv
            return dict(rec), {k: v.grad for k, v in s.items() if v.grad is not None}
        cap = Kinks()
        r32, g32 = run(torch.float32, cap)
        r64, g64 = run(torch.float64, Kinks(cap.relu, cap.pool))
        li = 17
        y64 = r64[li]["x"]                                  # NCHW pre-norm output
        gb64 = r64[li]["gbn"]                               # grad wrt the BN output (ReLU mask applied)
        rm, rv = sd[LAYER + ".1.running_mean"].double(), sd[LAYER + ".1.running_var"].double()
        inv = 1.0 / torch.sqrt(rv + 1e-5)
        xh64 = (y64 - rm[None, :, None, None]) * inv[None, :, None, None]
        dgam64 = (gb64 * xh64).sum((0, 2, 3))
        yh = torch.from_numpy(d[math + "_y"]).double().reshape(B, H, H, NF).permute(0, 3, 1, 2)
        gh_all = torch.from_numpy(d[math + "_g"]).double().reshape(B, H, H, 2 * NF)[..., :NF].permute(0, 3, 1, 2)
        # HIP's g is the gradient wrt the ReLU output: apply HIP's mask (z > 0 with z = BN(y) in fp32)
        gam, bet = sd[LAYER + ".1.weight"].double(), sd[LAYER + ".1.bias"].double()
        zh = gam[None, :, None, None] * (yh - rm[None, :, None, None]) * inv[None, :, None, None] + bet[None, :, None, None]
        gh = gh_all * (zh > 0)
        xhh = (yh - rm[None, :, None, None]) * inv[None, :, None, None]

        def rel(a, b):
            return ((a - b).norm() / b.norm()).item()
        print(f"[{math}] y rel {rel(yh, y64):.2e}  g_pre rel {rel(gh, gb64):.2e}")
        print(f"   dgamma: HIP {rel(torch.from_numpy(d[math + '_dgamma']).double(), g64[LAYER + '.1.weight'].double()):.2e}"
              f"  fp32-ref {rel(g32[LAYER + '.1.weight'].double(), g64[LAYER + '.1.weight'].double()):.2e}")
        print(f"   dgamma from HIP g & y summed in fp64 {rel((gh * xhh).sum((0, 2, 3)), dgam64):.2e};"
              f" from exact g, HIP y {rel((gb64 * xhh).sum((0, 2, 3)), dgam64):.2e};"
              f" from HIP g, exact y {rel((gh * xh64).sum((0, 2, 3)), dgam64):.2e}")
        eg = gh - gb64
        print(f"   g error: mean/rms {(eg.mean() / eg.pow(2).mean().sqrt()).item():+.3f};"
              f" corr with xhat {(eg * xh64).sum().item() / (eg.norm() * xh64.norm()).item():+.4f}")
        per = ((eg * xh64).sum((0, 2, 3)) / dgam64.abs().clamp_min(1e-300))
        print("   per-channel dgamma error from g:", " ".join(f"{v:+.1e}" for v in per.tolist()))
        if math + "_dyO" in d.files:
            dyo64 = conv_rec["dyO"]                                   # NCHW fp64 (HIP's branch)
            dyoh = torch.from_numpy(d[math + "_dyO"]).double().reshape(B, H, H, NF).permute(0, 3, 1, 2)
            w0 = conv_rec["w"].double()
            # g wrt out.0's input recomputed in fp64 from HIP's dyO: the first n_feat channels are g of this layer
            gi = torch.nn.grad.conv2d_input((B, 2 * NF, H, H), w0, dyoh, padding=1)[:, :NF] * (zh > 0)
            print(f"   dyO rel {rel(dyoh, dyo64):.2e}; dgamma from fp64 dgrad of HIP's dyO "
                  f"{rel((gi * xh64).sum((0, 2, 3)), dgam64):.2e}; HIP dgrad vs fp64 dgrad of HIP's dyO {rel(gh, gi):.2e},"
                  f" dgamma from that dgrad error {rel(((gh - gi) * xh64).sum((0, 2, 3)) + dgam64, dgam64):.2e}")


if __name__ == "__main__":
    if sys.argv[1] == "--analyse":
        analyse(sys.argv[2])
    else:
        run_box(sys.argv[1])
