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


@pytest.mark.parametrize("n,bs,world", [(65, 32, 2), (64, 32, 2), (63, 32, 2), (100, 7, 3), (13500, 32, 8),
                                        (5, 32, 8), (1, 4, 1), (47, 5, 4)])
def test_shard_epoch_same_step_count_on_every_rank(n, bs, world):
    """order[rank::world] + per-rank batching gave ranks different step counts (train=65, bs=32,
    world=2: 2 vs 1 steps) and the rank with the extra step hung in its all-reduce.  shard_epoch: equal step
    counts, disjoint near-equal parts per global batch, every sample used except < world of a ragged tail."""
    import sys
    sys.path.insert(0, ROOT)
    from cdm_amd.trainer import shard_epoch
    order = torch.randperm(n, generator=torch.Generator().manual_seed(n))
    per = [shard_epoch(order, bs, world, r) for r in range(world)]
    steps = {len(p) for p in per}
    assert len(steps) == 1
    used = []
    for j in range(len(per[0])):
        parts = [per[r][j][0] for r in range(world)]
        counts = {per[r][j][1] for r in range(world)}
        assert len(counts) == 1 and counts.pop() == sum(len(p) for p in parts)
        sizes = [len(p) for p in parts]
        assert max(sizes) - min(sizes) <= 1 and min(sizes) >= 1 and max(sizes) <= bs
        used.extend(torch.cat(parts).tolist())
    assert len(used) == len(set(used))
    assert n - world < len(used) <= n
    assert used == order[:len(used)].tolist()          # one pass over the epoch's permutation, in order


def _ragged_worker(rank, world, port, out, sizes):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)
    import cdm_amd  # noqa: F401
    from cdm_amd.trainer import GradBucketer, backward_order
    total = sum(sizes)
    names, grads = _rank_sq_grads(rank, sizes, grad_numel=total * 64 * 64 / world)
    order = backward_order(names)
    flat = torch.cat([grads[n].reshape(-1) for _, grp in order for n in grp])
    ranges, off = {}, 0
    for st, grp in order:
        k = sum(grads[n].numel() for n in grp)
        ranges[st] = (off, off + k); off += k
    bk = GradBucketer(flat, ranges)
    for st, _ in order:
        bk.stage_ready(st)
    bk.wait()
    if rank == 0:
        torch.save(flat / world, out)                  # the Trainer's Adam applies the 1/world scale
    dist.barrier()
    dist.destroy_process_group()


def _rank_sq_grads(rank, sizes, grad_numel, nf=8, T=50):
    """Oracle gradient of sum (pred - noise)^2 / grad_numel over this rank's samples (its own BN batch)."""
    from oracle import ref_cpu as R
    import cdm_amd
    torch.manual_seed(0)
    m = cdm_amd.ContextUnet(1, nf, 6, 64)
    sd = R.clone_sd(m.state_dict())
    keys = [k for k, _, kind in R.state_dict_layout(1, nf, 6, 64) if kind == "param"]
    for k in keys:
        sd[k].requires_grad_(True)
    B = sizes[rank]
    g = torch.Generator().manual_seed(300 + rank)
    x = torch.rand(B, 1, 64, 64, generator=g); noise = torch.randn(B, 1, 64, 64, generator=g)
    c = torch.rand(B, 6, generator=g); t = torch.randint(1, T + 1, (B,), generator=g)
    _, _, ab = R.make_schedule(T)
    w, b = R.draw_shortcut(1, nf)
    pred = R.unet_forward(sd, R.perturb_input(x, t, noise, ab), t / T, c, n_feat=nf, n_cfeat=6, height=64,
                          train=True, shortcut=(w, b))
    (((pred - noise) ** 2).sum() / grad_numel).backward()
    return [n for n, _ in m.named_parameters()], {k: sd[k].grad.detach().clone() for k in keys}


def test_ragged_global_batch_weighted_by_sample_count(tmp_path):
    """Ranks holding 3 and 2 samples of a 5-sample global batch: the Trainer's weighting (per-rank gradient
    scaled by 2 / (global_count * HW / world), summed by the bucketed all-reduce, times 1/world) equals the
    gradient of F.mse_loss over all 5 samples (each rank's forward on its own BatchNorm batch) — not the mean of
    the two per-rank means."""
    import sys
    sys.path.insert(0, ROOT)
    sizes = (3, 2)
    out = str(tmp_path / "flat.pt")
    mp.spawn(_ragged_worker, args=(2, _free_port(), out, sizes), nprocs=2, join=True)
    got = torch.load(out)
    import cdm_amd  # noqa: F401
    from cdm_amd.trainer import backward_order
    old = torch.get_num_threads()
    torch.set_num_threads(2)
    try:
        per = [_rank_sq_grads(r, sizes, grad_numel=sum(sizes) * 64 * 64) for r in range(2)]
    finally:
        torch.set_num_threads(old)
    names = per[0][0]
    order = backward_order(names)
    expect = torch.cat([(per[0][1][n] + per[1][1][n]).reshape(-1) for _, grp in order for n in grp])
    assert (got - expect).abs().max().item() <= 1e-6 * expect.abs().max().item()
    # the unweighted mean of per-rank means differs (3 vs 2 samples)
    means = [_rank_sq_grads(r, sizes, grad_numel=sizes[r] * 64 * 64) for r in range(2)]
    naive = torch.cat([((means[0][1][n] + means[1][1][n]) / 2).reshape(-1) for _, grp in order for n in grp])
    assert (naive - expect).abs().max().item() > 1e-3 * expect.abs().max().item()
