"""Exploratory timings of the BASELINE configs beyond C2 (one JSON line per measurement).

    python tools/probe_configs.py c4            # conv_math bf16/x3: train img/s, sample ms/step at w in {0,1,3}
    python tools/probe_configs.py c5 [B]        # 256x256, n_feat=256, T=2000: train + sample timings at batch B
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, n):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n


def run(nf, H, T, B, math, steps, sample_n, sample_steps, ws=(0.0,)):
    from cdm_amd import ContextUnet, Trainer
    from cdm_amd.diffusion import GraphSampler, Schedule
    torch.manual_seed(0)
    m = ContextUnet(1, nf, 6, H, shortcut_source="device", conv_math=math).cuda()
    tr = Trainer(m, 1e-5, T, B, seed=0, use_graph=True)
    g = torch.Generator(device="cuda").manual_seed(1234)
    x0 = torch.rand(B, 1, H, H, device="cuda", generator=g)
    c = torch.rand(B, 6, device="cuda", generator=g)
    for _ in range(2):
        tr.step(x0, c)
    dt = timed(lambda: tr.step(x0, c), steps)
    out = {"nf": nf, "H": H, "B": B, "math": math, "train_ms": dt * 1e3, "train_img_s": B / dt,
           "loss": float(tr.loss.item()), "mem_gb": torch.cuda.max_memory_allocated() / 1e9}
    del tr
    m.eval()
    sched = Schedule(T, "cuda")
    for w in ws:
        params = torch.rand(sample_n, 6, generator=torch.Generator().manual_seed(77))
        smp = GraphSampler(m, sched, sample_n, w, params, save_rate=20, z_source="device", seed=4321)
        smp.prepare_rng(host_z=False)
        xT = torch.randn(sample_n, 1, H, H, generator=torch.Generator().manual_seed(99))
        smp.prepare()
        smp.run(xT, steps=2)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        x = smp.run(xT, steps=sample_steps)[0]
        torch.cuda.synchronize()
        ds = (time.perf_counter() - t0) / sample_steps
        fin = bool(torch.isfinite(x).all())
        out[f"sample_w{w:g}_ms_per_step"] = ds * 1e3
        out[f"sample_w{w:g}_img_s_T"] = sample_n / (ds * T)
        out[f"sample_w{w:g}_finite"] = fin
        del smp
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    which = sys.argv[1]
    if which == "c4":
        maths = sys.argv[2].split(",") if len(sys.argv) > 2 else ["bf16", "x3", "x6"]
        for math in maths:
            run(128, 64, 1500, 256, math, 10, 256, 50, ws=(0.0, 1.0, 3.0))
    elif which == "c5":
        B = int(sys.argv[2]) if len(sys.argv) > 2 else 4
        math = sys.argv[3] if len(sys.argv) > 3 else "x6"
        run(256, 256, 2000, B, math, 3, B, 10)
