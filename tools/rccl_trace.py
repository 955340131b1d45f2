"""RCCL readiness trace: the Trainer's data-parallel path (force_ddp) in a one-rank "nccl" process group on the one-GPU
box, n_feat=128, bs=64, a few steps — run under rocprofv3 --kernel-trace, then summarised by tools/rccl_timeline.py:

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3_rccl -o rccl -- python3 tools/rccl_trace.py
"""
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    import cdm_amd
    torch.manual_seed(0)
    m = cdm_amd.ContextUnet(1, 128, 6, 64, shortcut_source="device").cuda()
    B = 64
    tr = cdm_amd.Trainer(m, 1e-5, 1500, B, seed=0, force_ddp=True)
    g = torch.Generator(device="cuda").manual_seed(1234)
    x = torch.rand(B, 1, 64, 64, device="cuda", generator=g); c = torch.rand(B, 6, device="cuda", generator=g)
    stages = []
    tr.stage_hook = lambda name: stages.append(name)
    for _ in range(4):
        tr.step(x, c)
    torch.cuda.synchronize()
    print("stages per step:", stages[-7:], "loss", float(tr.loss.item()), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
