"""Timing ablations of the h3 LDS-halo conv (128->128 @64x64, B=256): where does the kernel's time go?

    python tools/conv_ablation.py            (GPU) -> one JSON line: ms per launch for each ablation

  0  shipped kernel            2  every MFMA issued twice (MFMA work x2, staging unchanged)
  1  fragment prefetch         4  B staged only for the first two groups (no per-group B traffic)
  8  halo without the split    12 = 4 + 8 (no B staging, no split)      14 = 12 + 2
  65 prefetch, 2 fragment reads per MFMA gap      129 prefetch, all reads after the tap's first MFMA
  bits 16+: tiles per block (1 | 8 << 16 = the shipped kernel at this shape: 8 256-pixel tiles per block)
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(B=256, H=64, C=128, reps=10, relu=True):
    import cdm_amd
    L = cdm_amd.lib()
    s = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device="cuda").manual_seed(7)
    x = torch.randn(B * H * H, C, device="cuda", generator=g)
    if relu:
        x = x.relu()
    W = torch.randn(C, C, 3, 3, device="cuda", generator=g) * 0.05
    b = torch.zeros(C, device="cuda")
    wpk = torch.empty(9 * C, C, device="cuda")
    L.cdm_pack_conv3x3(W.data_ptr(), b.data_ptr(), C, C, None, None, None, None, 0.0, wpk.data_ptr(), None, None, 16, s)
    wx = torch.empty(9 * C // 16 * 3 * C * 16, dtype=torch.bfloat16, device="cuda")
    am = torch.empty(2, device="cuda")
    L.cdm_amax_f32(wpk.data_ptr(), 9 * C, C, C, am.data_ptr() + 4, 0, s)
    L.cdm_split_f16x2(wpk.data_ptr(), C, 9 * C, C, am.data_ptr() + 4, wx.data_ptr(), s)
    L.cdm_amax_f32(x.data_ptr(), B * H * H, C, C, am.data_ptr(), 0, s)
    y = torch.empty(B * H * H, C, device="cuda")
    out = {"relu_input": relu}
    st = torch.empty((B * H * H + 127) // 128, 2, C, device="cuda")
    prod = lambda: L.cdm_conv3x3_fwd_h3(x.data_ptr(), B, H, H, C, C, wx.data_ptr(), am.data_ptr(), am.data_ptr() + 4,
                                        b.data_ptr(), y.data_ptr(), C, C, 0, st.data_ptr(), C, 16, None, s)
    fns = {"prod": prod}
    abls = [int(a) for a in os.environ.get("CDM_ABLS", "").split(",") if a] or [1, 1 | 2 << 16, 1 | 4 << 16,
                                                                               1 | 8 << 16, 1 | 16 << 16, 61]
    for abl in abls:
        fns[abl] = (lambda abl=abl: L.cdm_conv3x3_halo_ablate(
            abl, x.data_ptr(), B, H, C, C, wx.data_ptr(), am.data_ptr(), am.data_ptr() + 4, y.data_ptr(), C, C, s))
    for f in fns.values():
        for _ in range(3):
            f()
    times = {k: [] for k in fns}
    for _round in range(5):                        # interleaved rounds: clock / thermal drift hits every variant
        for k, f in fns.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                f()
            e1.record()
            e1.synchronize()
            times[k].append(e0.elapsed_time(e1) / reps)
    for k, v in times.items():
        key = k if k == "prod" or k < 65536 else f"{k & 0xffff}/tpb{k >> 16}"
        out[key] = round(sorted(v)[len(v) // 2], 4)
    print(json.dumps(out))


if __name__ == "__main__":
    main(relu=True)

