"""Data-parallel Trainer on the GPU box: 2 ranks (gloo, both on cuda:0 — the box has one GPU).

Exercises the real Trainer DDP path — flat backward-ordered gradient buffer, stage hooks from the
engine's backward, asynchronous bucketed all_reduce, rank-0 parameter/buffer broadcast, Adam with
1/world gradient scaling — and checks:
  * the exchanged gradient equals the mean of the per-shard gradients computed by the single-GPU
    module path (same kernels, same injected noise / t / shortcut)   rel err <= 1e-5
  * both ranks hold identical parameters after the step.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NF, B, T = 16, 4, 100


def _free_port():
    s = socket.socket(); s.bind(("127.0.0.1", 0)); p = s.getsockname()[1]; s.close(); return p


def _shard(rank):
    g = torch.Generator().manual_seed(200 + rank)
    x = torch.rand(B, 1, 64, 64, generator=g); c = torch.rand(B, 6, generator=g)
    noise = torch.randn(B, 1, 64, 64, generator=g); t = torch.randint(1, T + 1, (B,), generator=g)
    sc = torch.rand(2 * NF, generator=g) * 2 - 1
    return x, c, noise, t, sc


def _worker(rank, world, port, outdir):
    import sys
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    import cdm_amd
    torch.manual_seed(0)
    m = cdm_amd.ContextUnet(1, NF, 6, 64).cuda()
    tr = cdm_amd.Trainer(m, 1e-3, T, B, seed=0)
    assert tr.ddp and not tr.use_graph
    x, c, noise, t, sc = _shard(rank)
    tr.step(x.cuda(), c.cuda(), inject=(noise.cuda(), t.cuda().int(), sc.cuda()))
    torch.cuda.synchronize()
    torch.save({"g": (tr.gflat / world).cpu(), "p": tr.flat.cpu(), "ranges": tr.ranges}, os.path.join(outdir, f"r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_ddp_trainer_two_ranks(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    r0 = torch.load(tmp_path / "r0.pt"); r1 = torch.load(tmp_path / "r1.pt")
    assert torch.equal(r0["p"], r1["p"]), "ranks diverged"
    import cdm_amd
    from cdm_amd.trainer import backward_order
    import torch.nn.functional as F
    grads = []
    for rank in range(2):
        torch.manual_seed(0)
        m = cdm_amd.ContextUnet(1, NF, 6, 64).cuda().train()
        x, c, noise, t, sc = (v.cuda() for v in _shard(rank))
        m.draw_shortcut = lambda dev, n_sets=1, sc=sc: (sc[:NF].contiguous(), sc[NF:].contiguous())
        sched = cdm_amd.Schedule(T, "cuda")
        xp = cdm_amd.perturb_input(x, t, noise, sched)
        pred = m(xp, t.float() / T, c)
        F.mse_loss(pred, noise).backward()
        grads.append({n: p.grad.detach().cpu() for n, p in m.named_parameters()})
    order = backward_order(list(grads[0].keys()))
    expect = torch.cat([((grads[0][n] + grads[1][n]) / 2).reshape(-1) for _, grp in order for n in grp])
    err = (r0["g"] - expect).abs().max().item()
    assert err <= 1e-5 * expect.abs().max().item(), err
