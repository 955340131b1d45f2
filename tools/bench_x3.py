"""Accuracy and speed of the split-bf16 conv3x3 (cdm_conv3x3_fwd_x3) vs the fp32-MFMA conv (GPU box).

    python tools/bench_x3.py [--reps 10] [--rounds 3]

Accuracy: N=4 maps against an fp64 CPU conv (max |err| / max |ref| and relative L2) for the fp32 MFMA
path and nterm in {6, 3, 1}; inputs are ReLU'd normals (post-BN activations) and N(0, 0.03) weights.
Speed: interleaved HIP-event timing on the hot shapes at B=256.
"""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    import cdm_amd
    L = cdm_amd.lib()
    s = torch.cuda.current_stream().cuda_stream

    def pack(W, ci, co):
        b = torch.zeros(co, device="cuda")
        w = torch.empty(9 * ci, co, device="cuda")
        L.cdm_pack_conv3x3(W.data_ptr(), b.data_ptr(), ci, co, None, None, None, None, 0.0, w.data_ptr(), None, None,
                           16, s)
        wx = torch.empty(((9 * ci + 15) // 16) * 3 * co * 16, dtype=torch.bfloat16, device="cuda")
        L.cdm_split_bf16x3(w.data_ptr(), co, 9 * ci, co, wx.data_ptr(), s)
        return w, wx, b

    def run(mode, x, B, H, ci, co, w, wx, b, y):
        if mode == "f32":
            L.cdm_conv3x3_fwd(x.data_ptr(), B, H, H, ci, ci, w.data_ptr(), b.data_ptr(), y.data_ptr(), co, co, 0,
                              None, 0, 16, s)
        else:
            L.cdm_conv3x3_fwd_x3(x.data_ptr(), B, H, H, ci, ci, wx.data_ptr(), b.data_ptr(), y.data_ptr(), co, co, 0,
                                 None, 0, 16, int(mode[1:]), s)

    def wgrad(mode, dy, x, B, H, ci, co, slab, sp):
        if mode == "f32":
            L.cdm_conv3x3_wgrad(dy.data_ptr(), co, co, x.data_ptr(), B, H, H, ci, ci, sp, slab.data_ptr(), s)
        else:
            L.cdm_conv3x3_wgrad_x3(dy.data_ptr(), co, co, x.data_ptr(), B, H, H, ci, ci, sp, slab.data_ptr(),
                                   int(mode[1:]), s)

    modes = ["f32", "x6", "x3", "x1"]
    # ---- accuracy ----
    for (B, H, ci, co) in [(4, 64, 128, 128), (4, 32, 256, 256)]:
        g = torch.Generator().manual_seed(0)
        x = torch.relu(torch.randn(B, H, H, ci, generator=g))
        W = torch.randn(co, ci, 3, 3, generator=g) * 0.03
        ref = F.conv2d(x.permute(0, 3, 1, 2).double(), W.double(), padding=1).permute(0, 2, 3, 1).reshape(-1, co)
        w, wx, b = pack(W.cuda(), ci, co)
        xc = x.cuda().reshape(-1, ci).contiguous()
        y = torch.empty(B * H * H, co, device="cuda")
        for mode in modes:
            run(mode, xc, B, H, ci, co, w, wx, b, y)
            torch.cuda.synchronize()
            d = y.double().cpu() - ref
            print(f"acc {H}x{H} {ci}->{co} {mode}: max|err|/max|ref| {d.abs().max().item() / ref.abs().max().item():.3e}"
                  f"  relL2 {d.norm().item() / ref.norm().item():.3e}", flush=True)
        # weight gradient against fp64
        gy = torch.randn(B, H, H, co, generator=g)
        gref = torch.einsum("bhwo,bhwct->oct", gy.double(),
                            F.unfold(x.permute(0, 3, 1, 2).double(), 3, padding=1).reshape(B, ci, 9, H, H)
                            .permute(0, 3, 4, 1, 2)).reshape(co, 9 * ci)
        # slab layout is [co][tap*ci+ci] -> compare in that order
        gref = gref.reshape(co, ci, 9).permute(0, 2, 1).reshape(co, 9 * ci)
        sp = L.raw("cdm_gemm_splits")(B * H * H, 8)
        slab = torch.empty(sp, co, 9 * ci, device="cuda")
        for mode in modes:
            wgrad(mode, gy.cuda().reshape(-1, co).contiguous(), xc, B, H, ci, co, slab, sp)
            torch.cuda.synchronize()
            d = slab.double().sum(0).cpu() - gref
            print(f"acc wgrad {H}x{H} {ci}->{co} {mode}: max|err|/max|ref| "
                  f"{d.abs().max().item() / gref.abs().max().item():.3e}  relL2 {d.norm().item() / gref.norm().item():.3e}",
                  flush=True)
    # ---- speed ----
    shapes = [(256, 64, 128, 128), (256, 64, 256, 128), (256, 32, 256, 256), (256, 32, 128, 256)]
    bufs = {}
    for (B, H, ci, co) in shapes:
        g = torch.Generator(device="cuda").manual_seed(1)
        x = torch.relu(torch.randn(B * H * H, ci, device="cuda", generator=g))
        W = torch.randn(co, ci, 3, 3, device="cuda", generator=g) * 0.03
        bufs[(B, H, ci, co)] = (x, *pack(W, ci, co), torch.empty(B * H * H, co, device="cuda"))
    res, slabs = {}, {}
    for _ in range(a.rounds):
        for shp, (x, w, wx, b, y) in bufs.items():
            B, H, ci, co = shp
            flops = 2.0 * B * H * H * ci * co * 9
            for mode in modes:
                run(mode, x, *shp, w, wx, b, y); run(mode, x, *shp, w, wx, b, y)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    run(mode, x, *shp, w, wx, b, y)
                e1.record(); e1.synchronize()
                ms = e0.elapsed_time(e1) / a.reps
                res.setdefault((shp, mode), []).append((ms, flops / ms / 1e9))
        for shp, (x, w, wx, b, y) in bufs.items():
            B, H, ci, co = shp
            flops = 2.0 * B * H * H * ci * co * 9
            tiles = -(-co // 128) * -(-(9 * ci) // 128)            # engine.wgrad_splits: ~2048 workgroups
            sp = L.raw("cdm_gemm_splits")(B * H * H, max(1, min(512, -(-2048 // tiles))))
            slab = slabs.setdefault(shp, torch.empty(sp, co, 9 * ci, device="cuda"))
            for mode in modes:
                wgrad(mode, y, x, B, H, ci, co, slab, sp)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    wgrad(mode, y, x, B, H, ci, co, slab, sp)
                e1.record(); e1.synchronize()
                ms = e0.elapsed_time(e1) / a.reps
                res.setdefault((("wgrad",) + shp, mode), []).append((ms, flops / ms / 1e9))
    for (shp, mode), v in sorted(res.items(), key=str):
        v = sorted(v)
        ms, tf = v[len(v) // 2]
        print(f"speed {shp} {mode}: {ms:.3f} ms  {tf:.1f} TF/s (fp32-equivalent)")


if __name__ == "__main__":
    main()
