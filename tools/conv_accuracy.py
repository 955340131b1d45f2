"""Error of each conv3x3 arithmetic vs an fp64 conv (relative L2), next to torch's fp32 CPU conv.

    python tools/conv_accuracy.py        (GPU)  -> one JSON line per (shape, pass)
"""
import json
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import cdm_amd
    import test_gpu_kernels as T
    L = cdm_amd.lib()
    for (N, H, Cin, Cout) in [(1, 64, 128, 128), (2, 32, 256, 128), (4, 16, 256, 256)]:
        torch.manual_seed(4)
        x = torch.randn(N, Cin, H, H).relu(); W = torch.randn(Cout, Cin, 3, 3) * 0.05; b = torch.randn(Cout)
        gy = torch.randn(N, Cout, H, H) * 1e-6
        xd, Wd = x.double().requires_grad_(), W.double().requires_grad_()
        r64 = F.conv2d(xd, Wd, b.double(), padding=1); r64.backward(gy.double())
        xf, Wf = x.clone().requires_grad_(), W.clone().requires_grad_()
        r32 = F.conv2d(xf, Wf, b, padding=1); r32.backward(gy)
        refs = {"y": r64.detach(), "dx": xd.grad, "dW": Wd.grad}
        res = {"torch_fp32": dict(zip(refs, (r32.detach(), xf.grad, Wf.grad)))}
        res["h3"] = dict(zip(refs, T._conv_h3(L, x, W, b, gy, 16)))
        for nterm, name in ((6, "x6"), (3, "x3"), (1, "bf16")):
            Wc, bc = W.cuda(), b.cuda()
            wpk, wdg = T._pack3x3(L, Wc, bc, 16)
            wx, wdx = T._split(L, wpk, 9 * Cin, Cout), T._split(L, wdg, 9 * Cout, Cin)
            xn, gyn = T._nhwc(x), T._nhwc(gy)
            y = torch.empty(N * H * H, Cout, device="cuda")
            L.cdm_conv3x3_fwd_x3(xn.data_ptr(), N, H, H, Cin, Cin, wx.data_ptr(), bc.data_ptr(), y.data_ptr(), Cout,
                                 Cout, 0, None, 0, 16, nterm, T._s())
            dx = torch.empty(N * H * H, Cin, device="cuda")
            L.cdm_conv3x3_fwd_x3(gyn.data_ptr(), N, H, H, Cout, Cout, wdx.data_ptr(), None, dx.data_ptr(), Cin, Cin, 0,
                                 None, 0, 16, nterm, T._s())
            sp = L.raw("cdm_gemm_splits")(N * H * H, 5)
            slab = torch.empty(sp, Cout, 9 * Cin, device="cuda")
            L.cdm_conv3x3_wgrad_x3(gyn.data_ptr(), Cout, Cout, xn.data_ptr(), N, H, H, Cin, Cin, sp, slab.data_ptr(),
                                   nterm, T._s())
            dW = torch.empty(Cout, Cin, 3, 3, device="cuda")
            L.cdm_slab_reduce(slab.data_ptr(), sp, Cout, 9 * Cin, dW.data_ptr(), 9 * Cin, 1, 9, Cin, 0, 1.0, T._s())
            torch.cuda.synchronize()
            res[name] = {"y": T._nchw(y, N, H, H, Cout), "dx": T._nchw(dx, N, H, H, Cin), "dW": dW}
        out = {"shape": [N, H, Cin, Cout]}
        for k, r in refs.items():
            out[k] = {m: float((v[k].double().cpu() - r).norm() / r.norm()) for m, v in res.items()}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
