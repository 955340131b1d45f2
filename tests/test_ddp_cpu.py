"""Data-parallel gradient exchange on CPU with gloo, world_size 2 (runs in the build container).

Each rank computes the CPU-oracle gradient of ContextUnet (n_feat=8) on its own shard, lays it out in
the Trainer's flat backward-completion order, and exchanges it with the Trainer's GradBucketer
(stage buckets, async all_reduce).  After the exchange every rank must hold sum_r grad_r, which is
world * (mean of the per-shard gradients) — the data-parallel training semantics of SURVEY §8e.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket(); s.bind(("127.0.0.1", 0)); p = s.getsockname()[1]; s.close(); return p


def _shard_grads(rank, nf=8, B=2, T=50):
    from oracle import ref_cpu as R
    import cdm_amd
    torch.manual_seed(0)
    m = cdm_amd.ContextUnet(1, nf, 6, 64)
    sd = R.clone_sd(m.state_dict())
    g = torch.Generator().manual_seed(100 + rank)
    x = torch.rand(B, 1, 64, 64, generator=g); noise = torch.randn(B, 1, 64, 64, generator=g)
    c = torch.rand(B, 6, generator=g); t = torch.randint(1, T + 1, (B,), generator=g)
    _, _, ab = R.make_schedule(T)
    tr = R.OracleTrainer(sd, n_feat=nf, n_cfeat=6, height=64)
    torch.manual_seed(7 + rank)
    _, _, grads = tr.step(x, c, noise, t, T, ab, lambda: R.draw_shortcut(1, nf))
    return m, grads


def _worker(rank, world, port, out):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)
    import cdm_amd  # noqa: F401
    from cdm_amd.trainer import GradBucketer, backward_order
    m, grads = _shard_grads(rank)
    order = backward_order([n for n, _ in m.named_parameters()])
    flat = torch.cat([grads[n].reshape(-1) for _, grp in order for n in grp])
    ranges, off = {}, 0
    for st, grp in order:
        k = sum(grads[n].numel() for n in grp)
        ranges[st] = (off, off + k); off += k
    bk = GradBucketer(flat, ranges)
    for st, _ in order:                    # stage completion order of the engine's backward
        bk.stage_ready(st)
    bk.wait()
    if rank == 0:
        torch.save(flat, out)
    dist.barrier()
    dist.destroy_process_group()


def test_bucketed_allreduce_equals_mean_of_shards(tmp_path):
    import sys
    sys.path.insert(0, ROOT)
    import cdm_amd  # noqa: F401
    from cdm_amd.trainer import backward_order
    out = str(tmp_path / "flat.pt")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    reduced = torch.load(out)
    old = torch.get_num_threads()
    torch.set_num_threads(2)                 # same intra-op split as the workers: identical fp32 sums
    try:
        m, g0 = _shard_grads(0)
        _, g1 = _shard_grads(1)
    finally:
        torch.set_num_threads(old)
    order = backward_order([n for n, _ in m.named_parameters()])
    expect = torch.cat([(g0[n] + g1[n]).reshape(-1) for _, grp in order for n in grp])
    err = (reduced - expect).abs().max().item()
    assert err <= 1e-6 * expect.abs().max().item(), err


def test_backward_order_covers_every_parameter_once():
    import sys
    sys.path.insert(0, ROOT)
    import cdm_amd
    from cdm_amd.trainer import backward_order
    m = cdm_amd.ContextUnet(1, 16, 6, 64)
    names = [n for n, _ in m.named_parameters()]
    flat = [n for _, grp in backward_order(names) for n in grp]
    assert sorted(flat) == sorted(names) and len(flat) == len(set(flat))
    # up0 (67 MB at n_feat=128) must complete before the encoder so its all-reduce overlaps it
    stages = [st for st, _ in backward_order(names)]
    assert stages.index("up0emb") < stages.index("down2") < stages.index("init")
