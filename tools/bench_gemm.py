"""Interleaved A/B timing of the conv GEMM variants on the hot shapes (GPU box).

    python tools/bench_gemm.py [--rounds 5] [--reps 10]
Reports TFLOP/s per (shape, variant): median and best over interleaved rounds.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--variants", default="0,2,3,4")
    a = ap.parse_args()
    import cdm_amd
    L = cdm_amd.lib()
    s = torch.cuda.current_stream().cuda_stream
    shapes = [(256, 64, 128, 128), (256, 32, 256, 256), (256, 64, 256, 128), (256, 32, 128, 128), (256, 32, 128, 256)]
    variants = [int(v) for v in a.variants.split(",")]
    res = {}
    bufs = {}
    for (B, H, ci, co) in shapes:
        g = torch.Generator(device="cuda").manual_seed(1)
        x = torch.randn(B * H * H, ci, device="cuda", generator=g)
        W = torch.randn(co, ci, 3, 3, device="cuda", generator=g) * 0.05
        b = torch.zeros(co, device="cuda")
        w = torch.empty(9 * ci, co, device="cuda"); wkc = torch.empty(9 * ci, co, device="cuda")
        L.cdm_pack_conv3x3(W.data_ptr(), b.data_ptr(), ci, co, None, None, None, None, 0.0, w.data_ptr(), None, None,
                           0, s)
        L.cdm_pack_conv3x3(W.data_ptr(), b.data_ptr(), ci, co, None, None, None, None, 0.0, wkc.data_ptr(), None, None,
                           16, s)
        y = torch.empty(B * H * H, co, device="cuda")
        st = torch.empty((B * H * H + 127) // 128, 2, co, device="cuda")
        bufs[(B, H, ci, co)] = (x, (w, wkc), b, y, st)
    for r in range(a.rounds):
        for shp, (x, ws, b, y, st) in bufs.items():
            B, H, ci, co = shp
            flops = 2.0 * B * H * H * ci * co * 9
            ref = None
            for v in variants:
                w = ws[1] if v in (3, 4) else ws[0]

                def go():
                    L.cdm_conv3x3_fwd_variant(v, x.data_ptr(), B, H, H, ci, ci, w.data_ptr(), b.data_ptr(),
                                              y.data_ptr(), co, co, 0, st.data_ptr(), co, s)
                go(); go()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    go()
                e1.record(); e1.synchronize()
                ms = e0.elapsed_time(e1) / a.reps
                res.setdefault((shp, v), []).append(flops / ms / 1e9)
                if ref is None:
                    ref = y.clone()
                else:
                    d = (y - ref).abs().max().item() / ref.abs().max().item()
                    assert d < 1e-5, f"variant {v} disagrees with variant {variants[0]}: {d}"
    for (shp, v), tf in sorted(res.items()):
        tf = sorted(tf)
        print(f"B{shp[0]} {shp[1]}x{shp[1]} {shp[2]}->{shp[3]} variant {v}: median {tf[len(tf)//2]:.1f} TF/s best {tf[-1]:.1f}")


if __name__ == "__main__":
    main()
