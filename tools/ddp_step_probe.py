"""Per-rank cost of the data-parallel train step on one GPU: the C2 step through Trainer(force_ddp=True) in a one-rank
RCCL group (eager launches, stage-bucketed async all-reduce, Adam after the bucket wait — the path every rank of an
N > 1 bench run takes) against the hipGraph-replayed single-GPU step, same seeds; also the host time to issue one eager
step (launches only, no wait).  The gap between the two is what data parallelism costs before any inter-GPU traffic.

    python tools/ddp_step_probe.py [steps]         (GPU box; MASTER_ADDR=127.0.0.1 set here)
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(ddp: bool, steps: int):
    import bench
    from cdm_amd import ContextUnet, Trainer
    torch.manual_seed(0)
    model = ContextUnet(1, bench.NF, bench.NCF, bench.H, shortcut_source="device", conv_math="h3").cuda()
    tr = Trainer(model, 1e-5, bench.T, 256, seed=0, use_graph=not ddp, force_ddp=ddp)
    g = torch.Generator(device="cuda").manual_seed(1234)
    x0 = torch.rand(256, 1, bench.H, bench.H, device="cuda", generator=g)
    c = torch.rand(256, bench.NCF, device="cuda", generator=g)
    for _ in range(3):
        tr.step(x0, c)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr.step(x0, c)
    issue = time.perf_counter() - t0          # host time to issue one step (the GPU is idle at its start)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        tr.step(x0, c)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    loss = float(tr.loss.item())
    del tr, model
    torch.cuda.empty_cache()
    return {"ms_per_step": round(ms, 3), "host_issue_ms": round(issue * 1e3, 3), "loss": loss}


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29531")
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    out = {"graph_single_gpu": run(False, steps), "ddp_one_rank_rccl": run(True, steps)}
    out["ddp_over_graph"] = round(out["ddp_one_rank_rccl"]["ms_per_step"] / out["graph_single_gpu"]["ms_per_step"], 4)
    print(json.dumps(out))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
