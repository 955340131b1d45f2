"""The Trainer's data-parallel path over RCCL (torch.distributed backend "nccl") on the one-GPU box.

A one-rank "nccl" process group with Trainer(force_ddp=True) runs exactly the code the N > 1 bench runs — rank-0
parameter / BatchNorm-buffer broadcasts, the engine's stage hooks enqueueing asynchronous all_reduce calls on RCCL's
stream for each backward-completion slice of the flat gradient buffer, GradBucketer.wait() ordering Adam after every
collective — at n_feat=128 (every fused BN-backward layer live).  With one rank a SUM all-reduce is the identity, so
the step must equal the plain single-GPU Trainer step bit for bit: parameters, Adam moments, gradients, BN running
statistics and loss, over two steps with an LR change.  (The scaling number is the driver's 8-GPU run; this is
readiness evidence: RCCL initialised and exercised on MI355X.)
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NF, B, T = 128, 8, 1500


def _free_port():
    s = socket.socket(); s.bind(("127.0.0.1", 0)); p = s.getsockname()[1]; s.close(); return p


def _run(cdm_amd, ddp):
    torch.manual_seed(0)
    m = cdm_amd.ContextUnet(1, NF, 6, 64).cuda()
    m.shortcut_source = "device"
    tr = cdm_amd.Trainer(m, 1e-3, T, B, seed=3, force_ddp=ddp, use_graph=False)
    assert tr.ddp == ddp
    g = torch.Generator().manual_seed(41)
    x = torch.rand(B, 1, 64, 64, generator=g).cuda(); c = torch.rand(B, 6, generator=g).cuda()
    losses = []
    for k in range(2):
        if k == 1:
            tr.set_lr(5e-4)
        losses.append(float(tr.step(x, c).item()))
    torch.cuda.synchronize()
    return {"p": tr.flat.cpu(), "g": tr.gflat.cpu(), "m": tr.m.cpu(), "v": tr.v.cpu(), "bn": tr.bnflat.cpu(),
            "loss": losses}


def _worker(rank, world, port, outdir):
    import sys
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    assert dist.get_backend() == "nccl"
    import cdm_amd
    out = {"ddp": _run(cdm_amd, True), "plain": _run(cdm_amd, False)}
    # the collective itself moved data: an all_reduce of a known tensor through the same group
    t = torch.arange(1000, dtype=torch.float32, device="cuda")
    w = dist.all_reduce(t, async_op=True)
    w.wait()
    out["probe"] = t.cpu()
    torch.save(out, os.path.join(outdir, "rccl.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_trainer_ddp_path_over_rccl_single_rank(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    mp.spawn(_worker, args=(1, _free_port(), str(tmp_path)), nprocs=1, join=True)
    r = torch.load(tmp_path / "rccl.pt")
    a, b = r["ddp"], r["plain"]
    for k in ("p", "g", "m", "v", "bn"):
        assert torch.equal(a[k], b[k]), k
    assert a["loss"] == b["loss"]
    assert torch.equal(r["probe"], torch.arange(1000, dtype=torch.float32))
