"""Per-shape rates of the h3 LDS-halo conv (forward, ReLU'd randn input like the forward's real operands):
every 3x3 conv shape of the C2 network at B=256 (and B=512, the CFG batch), HIP-event timed.

    python tools/conv_shapes.py        (GPU) -> one JSON line per shape: ms per launch, fp32-equivalent TF/s
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [(64, 128, 128), (64, 256, 128), (32, 128, 256), (32, 256, 256), (32, 128, 128), (32, 256, 128)]


def rate(L, B, H, Cin, Cout, reps=10):
    s = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device="cuda").manual_seed(7)
    x = torch.randn(B * H * H, Cin, device="cuda", generator=g).relu()
    W = torch.randn(Cout, Cin, 3, 3, device="cuda", generator=g) * 0.05
    b = torch.zeros(Cout, device="cuda")
    wpk = torch.empty(9 * Cin, Cout, device="cuda")
    L.cdm_pack_conv3x3(W.data_ptr(), b.data_ptr(), Cin, Cout, None, None, None, None, 0.0, wpk.data_ptr(), None, None,
                       16, s)
    wx = torch.empty(9 * Cin // 16 * 3 * Cout * 16, dtype=torch.bfloat16, device="cuda")
    am = torch.zeros(2, device="cuda")
    L.cdm_amax_f32(wpk.data_ptr(), 9 * Cin, Cout, Cout, am.data_ptr() + 4, 0, s)
    L.cdm_split_f16x2(wpk.data_ptr(), Cout, 9 * Cin, Cout, am.data_ptr() + 4, wx.data_ptr(), s)
    L.cdm_amax_f32(x.data_ptr(), B * H * H, Cin, Cin, am.data_ptr(), 0, s)
    y = torch.empty(B * H * H, Cout, device="cuda")
    st = torch.empty((B * H * H + 127) // 128, 2, Cout, device="cuda")
    f = lambda: L.cdm_conv3x3_fwd_h3(x.data_ptr(), B, H, H, Cin, Cin, wx.data_ptr(), am.data_ptr(), am.data_ptr() + 4,
                                     b.data_ptr(), y.data_ptr(), Cout, Cout, 0, st.data_ptr(), Cout, 16, None, s)
    for _ in range(3):
        f()
    ts = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            f()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) / reps)
    ms = sorted(ts)[1]
    gf = 2 * 9 * Cin * Cout * H * H * B / 1e9
    return {"B": B, "H": H, "Cin": Cin, "Cout": Cout, "ms": round(ms, 4), "tflops": round(gf / ms, 1)}


def main():
    import cdm_amd
    L = cdm_amd.lib()
    for B in (256, 512):
        for H, Cin, Cout in SHAPES:
            print(json.dumps(rate(L, B, H, Cin, Cout)), flush=True)


if __name__ == "__main__":
    main()
