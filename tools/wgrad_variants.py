"""h3 conv3x3 weight gradient: kernel-row kernel (variant 0, shipped) vs per-tap kernel (1) vs generic split GEMM
(2) on the train step's shapes — agreement of the reduced gradients and interleaved-median ms per launch.

    python tools/wgrad_variants.py            (GPU) -> one JSON line per shape
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(B, S, cin, cout, reps=10, variants=(0, 3, 1)):
    import cdm_amd
    from cdm_amd.engine import wgrad_splits
    L = cdm_amd.lib()
    s = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device="cuda").manual_seed(11)
    x = torch.randn(B * S * S, cin, device="cuda", generator=g).relu()
    dy = torch.randn(B * S * S, cout, device="cuda", generator=g) * 1e-3
    am = torch.zeros(2, device="cuda")
    L.cdm_amax_f32(dy.data_ptr(), B * S * S, cout, cout, am.data_ptr(), 0, s)
    L.cdm_amax_f32(x.data_ptr(), B * S * S, cin, cin, am.data_ptr() + 4, 0, s)
    sp = wgrad_splits(B * S * S, cout, 9 * cin)
    slab = torch.empty(sp, cout, 9 * cin, device="cuda")
    outs = {}
    fns = {}
    for v in variants:
        fns[v] = (lambda v=v: L.cdm_conv3x3_wgrad_h3_variant(dy.data_ptr(), cout, cout, x.data_ptr(), B, S, S, cin, cin,
                                                             am.data_ptr(), am.data_ptr() + 4, sp, slab.data_ptr(), v, s))
        slab.fill_(float("nan"))
        fns[v]()
        outs[v] = slab.sum(0)
    ref = outs[variants[-1]]
    res = {"shape": f"B{B} {S}x{S} {cin}->{cout}", "splits": sp,
           "gflop": round(2 * B * S * S * 9 * cin * cout / 1e9, 1)}
    for v in variants:
        res[f"relmax_{v}_vs_{variants[-1]}"] = float((outs[v] - ref).abs().max() / ref.abs().max())
    times = {v: [] for v in fns}
    for _ in range(5):
        for v, f in fns.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                f()
            e1.record()
            e1.synchronize()
            times[v].append(e0.elapsed_time(e1) / reps)
    for v, t in times.items():
        ms = sorted(t)[len(t) // 2]
        res[f"ms_{v}"] = round(ms, 4)
        res[f"tflops_{v}"] = round(res["gflop"] / ms, 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    for shp in ((256, 64, 128, 128), (256, 32, 256, 256), (256, 32, 128, 256), (256, 32, 128, 128), (256, 64, 256, 128)):
        run(*shp)
