"""Time the residual BatchNorm apply (init_conv.conv2 of the C2 step: B 256, 64x64, 128 channels into the 256-wide catO
slice) for the C_in = 1 shortcut and the in_channels = 3 form, with HIP events (GPU box).

    python tools/apply_probe.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import cdm_amd
    lb = cdm_amd.lib()
    s = torch.cuda.current_stream()
    B, H, C = 256, 64, 128
    P = B * H * H
    y = torch.randn(P, C, device="cuda")
    sc, sh = torch.rand(C, device="cuda"), torch.randn(C, device="cuda")
    out = torch.empty(P, 2 * C, device="cuda")
    am = torch.zeros(1, device="cuda")
    res = {}
    for xc in (1, 3):
        cp = 1 if xc == 1 else 4
        x = torch.randn(P, cp, device="cuda")
        w, b = torch.randn(C * xc, device="cuda"), torch.randn(C, device="cuda")

        def launch():
            if xc == 1:
                lb.cdm_norm_apply_fwd(4 | 8, y.data_ptr(), C, B, H, H, C, sc.data_ptr(), sh.data_ptr(), 0, None, 0, None,
                                      0, x.data_ptr(), w.data_ptr(), b.data_ptr(), B, out.data_ptr(), 2 * C,
                                      am.data_ptr(), s.cuda_stream)
            else:
                lb.cdm_norm_apply_fwd_resid_c(8, y.data_ptr(), C, B, H, H, C, sc.data_ptr(), sh.data_ptr(), x.data_ptr(),
                                              cp, xc, w.data_ptr(), b.data_ptr(), B, out.data_ptr(), 2 * C,
                                              am.data_ptr(), s.cuda_stream)
        for _ in range(3):
            launch()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(20):
            launch()
        e1.record(s)
        e1.synchronize()
        ms = e0.elapsed_time(e1) / 20
        res[f"xc={xc}"] = {"us": round(ms * 1e3, 1), "GB/s": round(2 * P * C * 4 / (ms * 1e-3) / 1e9, 1)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
