"""Host enqueue time of the data-parallel train step vs its GPU time.

On N > 1 GPUs the Trainer runs eager (its stage all-reduce hooks are host calls between the backward's launches), so
the host issues every kernel of every step (~270 launches through ctypes) plus 7 all-reduces and a broadcast.  If that
host work per step approached the GPU step time, N > 1 would go host-bound unnoticed.  This probe runs the DDP path in
a one-rank `nccl` (RCCL) process group (Trainer(force_ddp=True), as tests/test_gpu_rccl.py) at the bench shape and
reports, per mode (DDP eager, plain eager, plain graph replay):
  host_ms   time for the host to return from Trainer.step (no synchronisation inside the timed region)
  gpu_ms    HIP-event time of the step on the stream
  wall_ms   back-to-back steps, wall time per step including the final synchronisation (the steady state)
and the launch count per step (HIP API trace is not needed: the engine's C-ABI calls are counted).

    python tools/ddp_host_probe.py [out.json]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

NF, NCF, H, B, T = 128, 6, 64, 256, 1500


def count_calls(lib):
    """Wrap every cdm_* entry point of the loaded library with a counter (host-side only)."""
    counts = {"n": 0}
    for name in list(lib.protos):
        fn = getattr(lib, name, None)
        if fn is None or not callable(fn):
            continue

        def wrap(f):
            def g(*a):
                counts["n"] += 1
                return f(*a)
            return g
        setattr(lib, name, wrap(fn))
    return counts


def run(mode, steps=10, warmup=3):
    from cdm_amd import ContextUnet, Trainer
    torch.manual_seed(0)
    m = ContextUnet(1, NF, NCF, H, shortcut_source="device").cuda()
    tr = Trainer(m, 1e-5, T, B, seed=0, use_graph=(mode == "graph"), force_ddp=(mode == "ddp"))
    g = torch.Generator(device="cuda").manual_seed(1234)
    x0 = torch.rand(B, 1, H, H, device="cuda", generator=g)
    c = torch.rand(B, NCF, device="cuda", generator=g)
    eager = mode != "graph"
    for _ in range(warmup):
        tr.step(x0, c, eager=eager)
    torch.cuda.synchronize()
    host = []
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(steps):
        h0 = time.perf_counter()
        tr.step(x0, c, eager=eager)
        host.append((time.perf_counter() - h0) * 1e3)
    e1.record()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e3 / steps
    gpu = e0.elapsed_time(e1) / steps
    # per-step GPU time alone (synchronised single steps)
    singles = []
    for _ in range(3):
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); tr.step(x0, c, eager=eager); b.record(); b.synchronize()
        singles.append(a.elapsed_time(b))
    del tr, m
    torch.cuda.empty_cache()
    host.sort()
    return {"mode": mode, "host_ms_median": host[len(host) // 2], "host_ms_max": host[-1],
            "gpu_ms_back_to_back": gpu, "wall_ms_per_step": wall, "gpu_ms_single_step_min": min(singles)}


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "r4_ddp_host_probe.json")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    import cdm_amd
    res = []
    for mode in ("ddp", "eager", "graph"):
        r = run(mode)
        res.append(r)
        print(json.dumps(r), flush=True)
    counts = count_calls(cdm_amd.lib())          # C-ABI calls of one eager DDP step (after the timed runs)
    r = run("ddp", steps=1, warmup=0)
    res.append({"c_abi_calls_per_ddp_step": counts["n"] / 4.0})  # 1 + 3 single steps
    dist.destroy_process_group()
    rec = {"what": "host enqueue vs GPU time per C2 train step (n_feat=128, B=256, h3); ddp = Trainer(force_ddp=True) in "
                   "a one-rank nccl (RCCL) group: eager, 7 stage all-reduces + a running-stat broadcast per step",
           "results": res}
    os.makedirs(os.path.dirname(out), exist_ok=True)
    json.dump(rec, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
