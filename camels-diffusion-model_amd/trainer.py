"""The DDPM training step (a8) on the HIP engine, single- or multi-GPU.

One step == code/train_diffusion_condition.py:216-230 (and code/train_diffusion.py:141-151):
    noise ~ N(0,1), t ~ U{1..T}, x_pert = perturb_input(x, t, noise), eps = ContextUnet(x_pert, t/T, c)
    (train-mode BatchNorm), loss = mse(eps, noise), backward, Adam(lr) step.

MI355X design:
  * parameters, gradients and Adam moments live in three flat fp32 buffers; the module's nn.Parameters
    are re-pointed to views of the flat parameter buffer (state_dict stays reference-compatible);
  * noise / timesteps / the per-forward random 1x1 shortcut come from on-device Philox keyed by a
    device step counter, so the whole step (repack -> forward -> mse -> backward -> Adam) is captured
    once in a hipGraph and replayed (single GPU);
  * data parallel: one process per GPU; each rank trains on its own shard of the global batch; the
    flat gradient buffer is laid out in backward-completion order and cut into stage buckets that are
    all-reduced (RCCL over xGMI) asynchronously as soon as the engine reports a stage complete, so the
    67 MB up0 gradient and everything after it overlaps the encoder's backward; BatchNorm running stats
    are broadcast from rank 0 each step (DDP broadcast_buffers semantics), batch statistics stay local
    to the rank (reference semantics at the local batch; no SyncBN in the reference).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch

from ._lib import lib
from .diffusion import Schedule

STAGES: Tuple[Tuple[str, Tuple[str, ...]], ...] = (
    ("out", ("out.",)), ("up2", ("up2.",)), ("up1", ("up1.",)),
    ("up0emb", ("up0.", "timeembed", "contextembed")),
    ("down2", ("down2.",)), ("down1", ("down1.",)), ("init", ("init_conv.",)),
)


def _p(t):
    return None if t is None else t.data_ptr()


def _s():
    return torch.cuda.current_stream().cuda_stream


def backward_order(names: List[str]):
    """Parameter names in gradient-completion order, grouped by stage: [(stage, [names])]."""
    out, seen = [], set()
    for st, prefixes in STAGES:
        grp = [n for n in names if n.startswith(prefixes)]
        seen.update(grp)
        out.append((st, grp))
    missing = [n for n in names if n not in seen]
    if missing:
        raise AssertionError(f"parameters without a stage: {missing}")
    return out


class GradBucketer:
    """Stage-bucketed asynchronous gradient all-reduce over a flat gradient buffer.

    Device-agnostic (works with gloo on CPU tensors for tests, RCCL on MI355X)."""

    def __init__(self, gflat: torch.Tensor, ranges: Dict[str, Tuple[int, int]], group=None):
        import torch.distributed as dist
        self.dist = dist
        self.gflat, self.ranges, self.group = gflat, ranges, group
        self.world = dist.get_world_size(group)
        self.pending = []

    def stage_ready(self, stage: str):
        lo, hi = self.ranges[stage]
        if hi > lo:
            self.pending.append(self.dist.all_reduce(self.gflat[lo:hi], op=self.dist.ReduceOp.SUM,
                                                     group=self.group, async_op=True))

    def wait(self):
        for w in self.pending:
            w.wait()
        self.pending = []


class Trainer:
    def __init__(self, model, lrate: float, timesteps: int, batch_size: int, seed: int = 0,
                 use_graph: bool = True, group=None, broadcast_buffers: bool = True, force_ddp: bool = False):
        """``force_ddp``: take the data-parallel path (stage-bucketed async all-reduce, rank-0 broadcasts, eager
        steps) even in a one-rank process group — RCCL readiness on a one-GPU box (tests/test_gpu_rccl.py)."""
        self.model = model
        eng, P = model._engine_and_params()
        self.eng = eng
        dev = P["out.3.weight"].device
        self.dev = dev
        self.B, self.T = int(batch_size), int(timesteps)
        self.H, self.nf, self.ncf = model.h, model.n_feat, model.n_cfeat
        self.group = group
        import torch.distributed as dist
        self.ddp = dist.is_available() and dist.is_initialized() and (dist.get_world_size(group) > 1 or force_ddp)
        self.world = dist.get_world_size(group) if self.ddp else 1
        self.seed = int(seed)
        # ---- flat parameter / gradient / moment buffers in backward-completion order ----
        names = model._param_names
        order = backward_order(names)
        params = dict(model.named_parameters())
        total = sum(params[n].numel() for _, g in order for n in g)
        self.flat = torch.empty(total, device=dev)
        self.gflat = torch.zeros(total, device=dev)
        self.m = torch.zeros(total, device=dev)
        self.v = torch.zeros(total, device=dev)
        self.views: Dict[str, torch.Tensor] = {}
        self.grads: Dict[str, torch.Tensor] = {}
        self.ranges: Dict[str, Tuple[int, int]] = {}
        off = 0
        for st, grp in order:
            lo = off
            for n in grp:
                p = params[n]
                k = p.numel()
                view = self.flat[off:off + k].view_as(p)
                view.copy_(p.data)
                p.data = view
                self.views[n] = view
                self.grads[n] = self.gflat[off:off + k].view_as(p)
                off += k
            self.ranges[st] = (lo, off)
        self.total = total
        # ---- BatchNorm running stats in one flat buffer (one broadcast per step under DDP) ----
        bufs = [(n, b) for n, b in model.named_buffers() if n.endswith(("running_mean", "running_var"))]
        self.bnflat = torch.empty(sum(b.numel() for _, b in bufs), device=dev)
        off = 0
        for n, b in bufs:
            mod = model.get_submodule(n.rsplit(".", 1)[0])
            view = self.bnflat[off:off + b.numel()]
            view.copy_(b)
            mod._buffers[n.rsplit(".", 1)[1]] = view
            off += b.numel()
        self.broadcast_buffers = broadcast_buffers
        if self.ddp:
            dist.broadcast(self.flat, 0, group=group)
            dist.broadcast(self.bnflat, 0, group=group)
            self.bucketer = GradBucketer(self.gflat, self.ranges, group)
        # ---- optimizer state on device (fp64, as torch keeps lr / step as Python floats):
        #      [lr, step, -step_size, sqrt(bc2)] + the host-evaluated bias-correction table ----
        self.betas, self.eps = (0.9, 0.999), 1e-8
        self.opt_state = torch.tensor([float(lrate), 0.0, 0.0, 1.0], dtype=torch.float64, device=dev)
        self.adam_bc = adam_bias_table(*self.betas).to(dev)
        self.nonfinite = torch.zeros(1, dtype=torch.int32, device=dev)   # steps with a NaN / inf loss
        # ---- step buffers (per batch size: the epoch's ragged last batch gets its own) ----
        self.sched = Schedule(self.T, dev)
        self.sc = torch.empty(2 * self.nf, device=dev)
        self.nb = 256
        self.partial = torch.empty(2 * self.nb, device=dev)
        self.loss = torch.zeros(1, device=dev)
        self.ctr = torch.zeros(1, dtype=torch.int32, device=dev)
        self._bufs: Dict[int, "_StepBufs"] = {}
        self._use(self.B)
        self.use_graph = bool(use_graph) and not self.ddp
        self.graph = None
        self.steps = 0
        self._inject = None
        self.stage_hook = None        # optional extra on_stage(name) callback (tests / tracing)
        self.grad_numel = None        # per-step override of the loss-mean count (data-parallel ragged batches)

    # -------------------------------------------------------------------------------------------
    def _use(self, B: int):
        b = self._bufs.get(B)
        if b is None:
            b = self._bufs[B] = _StepBufs(self.eng, B, self.H, self.ncf, self.dev)
        self.cur = b
        return b

    @property
    def x0(self):
        return self.cur.x0

    @property
    def c(self):
        return self.cur.c

    def P(self):
        _, P = self.model._engine_and_params()
        return P

    def set_lr(self, lr: float):
        """optim.param_groups[0]['lr'] = lr (code/train_diffusion_condition.py:213); exact Python-float lr."""
        self.opt_state[0:1].fill_(float(lr))

    def check_finite(self, reset: bool = True) -> int:
        """Number of steps since the last check whose loss was NaN / inf (SURVEY §5 failure guard).  One host sync:
        call it once per epoch, not per step."""
        n = int(self.nonfinite.item())
        if reset and n:
            self.nonfinite.zero_()
        return n

    def _body(self, s: int):
        lb = lib()
        sb = self.cur
        B, HW, nf = sb.B, self.H * self.H, self.nf
        P = self._P
        seed = self.seed * 1000003 + (self._rank() << 20)
        if self._inject is None:
            lb.cdm_philox_normal(_p(sb.noise), B * HW, seed, 0, _p(self.ctr), s)
            lb.cdm_philox_randint(_p(sb.t_int), B, 1, self.T, seed, 1 << 24, _p(self.ctr), s)
            lb.cdm_philox_uniform(_p(self.sc), 2 * nf, -1.0, 1.0, seed, 2 << 24, _p(self.ctr), s)
        else:                      # parity mode: caller-provided draws (eager only)
            noise, t_int, sc = self._inject
            sb.noise.copy_(noise.reshape(-1)); sb.t_int.copy_(t_int.reshape(-1))
            self.sc.copy_(sc.reshape(-1))
        lb.cdm_perturb(_p(sb.x0), _p(sb.noise), _p(sb.t_int), None, 0, _p(self.sched.sab), _p(self.sched.omab), B, HW,
                       self.T, _p(sb.xpert), _p(sb.t_in), s)
        self.eng.repack(P, True, s)
        eps = self.eng.forward(sb.ws, P, sb.xpert, sb.t_in, sb.c, self.sc[:nf], self.sc[nf:], B, s)
        gnum = float(B * HW) if self.grad_numel is None else float(self.grad_numel)
        lb.cdm_mse(_p(eps), _p(sb.noise), B * HW, gnum, _p(sb.deps), _p(self.partial), self.nb, _p(self.loss),
                   _p(self.grads["out.3.bias"]), _p(self.nonfinite), s)
        hooks = [h for h in (self.bucketer.stage_ready if self.ddp else None, self.stage_hook) if h is not None]
        hook = (lambda name: [h(name) for h in hooks]) if hooks else None
        self.eng.backward(sb.ws, P, sb.deps, self.grads, s, out3_bias_done=True, on_stage=hook)
        if self.ddp:
            self.bucketer.wait()
        lb.cdm_adam(_p(self.flat), _p(self.gflat), _p(self.m), _p(self.v), self.total, _p(self.opt_state),
                    _p(self.adam_bc), self.adam_bc.shape[0], self.betas[0], self.betas[1], self.eps, 1.0 / self.world, s)
        lb.cdm_counter_add(_p(self.ctr), 1, s)

    def _rank(self):
        if not self.ddp:
            return 0
        import torch.distributed as dist
        return dist.get_rank(self.group)

    def _capture(self):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            self._body(torch.cuda.current_stream().cuda_stream)
        self.graph = g

    def step(self, x0: Optional[torch.Tensor] = None, c: Optional[torch.Tensor] = None, inject=None,
             global_count: Optional[int] = None, eager: bool = False) -> torch.Tensor:
        """One training step on batch (x0 [B,1,H,H] in [0,1], c [B, n_cfeat] or None = unconditional).

        ``inject=(noise [B,1,H,H], t [B] int, shortcut [2*n_feat] = weight|bias)`` replaces the on-device
        Philox draws for this step (parity testing; runs eagerly).
        ``global_count`` (data parallel): the number of samples all ranks process in this step when the ranks'
        batches differ in size; the gradient is then the mean over those samples (each rank weighted by its
        sample count, F.mse_loss over the union) instead of the mean of per-rank means."""
        self._inject = inject
        B = self.B if x0 is None else x0.shape[0]
        HW = self.H * self.H
        self.grad_numel = None if global_count is None else float(global_count) * HW / self.world
        sb = self._use(B)
        if x0 is not None:
            sb.x0.copy_(x0.reshape(B, self.H, self.H))
        if c is not None:
            sb.c.copy_(c.reshape(B, self.ncf))
        self._P = self.P()
        self.eng.invalidate()                 # the fused Adam updates parameters in place
        if self.ddp and self.broadcast_buffers:
            import torch.distributed as dist
            dist.broadcast(self.bnflat, 0, group=self.group)
        if self.use_graph and inject is None and B == self.B and self.grad_numel is None and not eager:
            if self.graph is None:
                self._body(_s())          # eager warm-up step (loads every kernel) then capture
                self._capture()
            else:
                self.graph.replay()
        else:
            self._body(_s())
        self.steps += 1
        return self.loss


def shard_epoch(order: torch.Tensor, batch_size: int, world: int, rank: int):
    """Data-parallel batches of one epoch for ``rank``: [(indices, global_count)], the same count of steps on
    every rank (a rank that ran an extra step would wait forever in its all-reduce).

    Global step j takes order[j*G : (j+1)*G] with G = batch_size * world (the reference's loop over one shuffled
    epoch, code/train_diffusion_condition.py:214-216, at a global batch of G) and splits it into ``world``
    contiguous near-equal parts (sizes differ by at most one).  ``global_count`` is that step's global batch size,
    passed to Trainer.step so the gradient is the mean over all its samples (each rank weighted by its sample
    count).  A last global batch with fewer samples than ranks is skipped (at most world - 1 samples of an epoch;
    the permutation differs every epoch)."""
    G = batch_size * world
    out = []
    for j in range(0, len(order), G):
        part = order[j:j + G]
        R = len(part)
        if R < world:
            break
        lo = rank * (R // world) + min(rank, R % world)
        n = R // world + (1 if rank < R % world else 0)
        out.append((part[lo:lo + n], R))
    return out


def adam_bias_table(beta1: float, beta2: float, n: int = 40960) -> torch.Tensor:
    """[n, 2] fp64: 1 - beta1**step and (1 - beta2**step)**0.5 for step = 1..n, evaluated with the Python-float
    expressions of torch.optim.Adam (_single_tensor_adam), so the device step size equals torch's bit for bit.
    The last row must be exactly (1, 1): later steps reuse it (both powers are below 2^-54 by then)."""
    rows = [(1 - beta1 ** float(s), (1 - beta2 ** float(s)) ** 0.5) for s in range(1, n + 1)]
    if rows[-1] != (1.0, 1.0):
        raise ValueError("bias-correction table too short for these betas")
    return torch.tensor(rows, dtype=torch.float64)


class _StepBufs:
    """Device buffers of one training step at batch size B (engine workspace included)."""

    def __init__(self, eng, B: int, H: int, ncf: int, dev):
        HW = H * H
        self.B = B
        self.x0 = torch.zeros(B, H, H, device=dev)
        self.c = torch.zeros(B, ncf, device=dev)
        self.noise = torch.empty(B * HW, device=dev)
        self.t_int = torch.empty(B, dtype=torch.int32, device=dev)
        self.t_in = torch.empty(B, device=dev)
        self.xpert = torch.empty(B, H, H, device=dev)
        self.deps = torch.empty(B, H, H, device=dev)
        self.ws = eng.workspace(B, True)
