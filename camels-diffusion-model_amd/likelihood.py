"""Likelihood / ELBO evaluation of a ContextUnet on the HIP engine.

Reference functions (same names, arguments and return values):
  calculate_likelihood(model, dataloader, timesteps, device, ab_t, b_t, a_t)
      code/train_diffusion_elbo.py:108-149  (identical copy: code/train_diffusion_paper.py:142-183)
      -> mean over samples of  sum_{t=1..T} mse_t / (2 b_t),  x_t = sqrt(ab) x + (1 - ab) noise
  calculate_elbo_and_bpd(model, dataloader, timesteps, device, ab_t, b_t, a_t)
      code/train_diffusion_paper.py:77-139  -> (avg_elbo, bpd): 10 evenly spaced t, sqrt(1 - ab) noise,
      weight 0.5 b/(1 - ab) for t > 1, divided by 10; bpd = elbo / (64*64 ln 2)
  calculate_elbo_and_bpd(x, pred_noise, noise, t, b_t, a_t, ab_t, dims)
      code/train_diffusion_elbo.py:74-105   -> (elbo, bpd) of one training batch (per-sample t)
The two same-named reference functions are told apart by their first argument (a model or a tensor).

The T-step NLL loop is the same shape as the sampler: per step a prologue (device step counter ->
t/T, shortcut row), a noise draw (on-device Philox, or a row of a pre-drawn table), the perturbation,
the full eval forward and a fused per-sample weighted-MSE accumulation.  K steps are captured in one
hipGraph and replayed; one graph per batch size (the last, ragged batch gets its own).

RNG (``noise_source``): "device" = noise on device, the per-forward 1x1 shortcut from the CPU RNG in the
reference GPU run's order; "host" = noise and shortcuts from the CPU RNG interleaved exactly as the
reference's CPU run draws them (noise_t, then the model's shortcut, for t = 1..T) — the parity mode.
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn as nn

from ._lib import lib
from .diffusion import Schedule


def _s():
    return torch.cuda.current_stream().cuda_stream


def _p(t):
    return None if t is None else t.data_ptr()


def _split_batch(item):
    if torch.is_tensor(item):
        return item, None
    x = item[0]
    c = item[1] if len(item) > 1 else None
    return x, c


class _EvalRun:
    """Device state of one batch size: inputs, noise, shortcut table, accumulator, step graph."""

    def __init__(self, ev: "LikelihoodEvaluator", B: int):
        self.ev, self.B = ev, B
        m = ev.model
        dev, H, nf, ncf = ev.dev, m.h, m.n_feat, m.n_cfeat
        T = ev.T
        E = lambda *sh: torch.empty(*sh, device=dev)
        self.HW = H * H
        self.x0 = E(B, self.HW)
        self.xt = E(B, H, H)
        self.cbuf = torch.zeros(B, ncf, device=dev)
        self.has_c = False
        self.acc = torch.zeros(B, device=dev)
        self.t_cur = E(1)
        self.cur_i = torch.zeros(1, dtype=torch.int32, device=dev)
        self.ctr = torch.zeros(1, dtype=torch.int32, device=dev)
        self.row = 2 * nf
        self.sc_table = E(T, self.row)
        self.sc_cur = E(self.row)
        host = ev.noise_source == "host"
        # host mode: noise table row (T - t) holds the draw for step t; device mode: one noise buffer
        self.noise = E(T if host else 1, B * self.HW)
        self.nstride = B * self.HW if host else 0
        self.ws = ev.eng.workspace(B, False)
        self.graph = None

    def step(self, s, mul, div, omab):
        ev, lb = self.ev, lib()
        lb.cdm_sample_prologue(_p(self.ctr), ev.T, _p(self.cur_i), _p(self.t_cur), _p(self.sc_table), self.row,
                               _p(self.sc_cur), s)
        self._body(s, mul, div, omab, self.nstride)

    def _body(self, s, mul, div, omab, nstride):
        ev, lb = self.ev, lib()
        B, HW, nf = self.B, self.HW, ev.model.n_feat
        if ev.noise_source == "device":
            lb.cdm_philox_normal(_p(self.noise), B * HW, ev.seed, 0, _p(ev.rng_ctr), s)
            lb.cdm_counter_add(_p(ev.rng_ctr), 1, s)
        lb.cdm_perturb(_p(self.x0), _p(self.noise), None, _p(self.cur_i), nstride, _p(ev.sched.sab), _p(omab),
                       B, HW, ev.T, _p(self.xt), None, s)
        eps = ev.eng.forward(self.ws, ev.P, self.xt, self.t_cur, self.cbuf if self.has_c else None,
                             self.sc_cur[:nf], self.sc_cur[nf:], B, s)
        if mul is not None:
            lb.cdm_mse_accum(_p(eps), _p(self.noise), nstride, ev.T, B, HW, None, _p(self.cur_i), _p(mul),
                             _p(div), _p(self.acc), s)

    def capture(self, K: int):
        ev = self.ev
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        rng = ev.rng_ctr.clone()
        with torch.cuda.stream(s):
            self.ctr.fill_(ev.T)
            self.step(s.cuda_stream, None, None, ev.sched.omab)     # warm-up: every kernel resident
            ev.rng_ctr.copy_(rng)                                   # ... without consuming a noise stream
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(K):
                self.step(torch.cuda.current_stream().cuda_stream, ev.nll_mul, ev.nll_div, ev.sched.omab)
        self.graph = g

    def load(self, x, c):
        B, dev = self.B, self.ev.dev
        self.x0.copy_(x.to(dev, torch.float32).reshape(B, self.HW))
        if self.has_c != (c is not None):
            self.graph = None                      # the captured forward reads (or skips) the context buffer
        self.has_c = c is not None
        if c is not None:
            self.cbuf.copy_(c.to(dev, torch.float32).reshape(B, -1))
        self.acc.zero_()


class LikelihoodEvaluator:
    """Holds the schedule tables, the per-batch-size runs and graphs of one model."""

    def __init__(self, model, timesteps: int, noise_source: str = "device", steps_per_graph: int = 10,
                 seed: int = 4321, use_graph: bool = True, sched_tensors=None):
        """``sched_tensors=(b_t, a_t, ab_t)``: the caller's schedule (the reference functions take them as
        arguments and use them as given); None builds the default schedule of the training scripts."""
        assert noise_source in ("device", "host")
        self.model, self.T = model, int(timesteps)
        self.eng, self.P = model._engine_and_params()
        self.dev = self.P["out.3.weight"].device
        self.sched = Schedule(self.T, self.dev, tensors=sched_tensors)
        self.noise_source = noise_source
        self.seed = seed
        self.K = max(1, int(steps_per_graph))
        self.use_graph = use_graph
        self.rng_ctr = torch.zeros(1, dtype=torch.int32, device=self.dev)
        b, _, ab = (v.cpu() for v in self.sched.tensors())
        # reference fp32 expressions, evaluated once into per-step tables
        self.nll_mul = torch.ones(self.T + 1, device=self.dev)
        self.nll_div = (2 * b).to(self.dev)                                   # elbo.py:140
        self.elbo_mul = (0.5 * (b / (1.0 - ab))).to(self.dev)                # paper.py:122
        self.elbo_div = torch.full((self.T + 1,), 10.0, device=self.dev)     # paper.py:124
        self.sqrt_omab = torch.sqrt(1 - ab).to(self.dev)                     # paper.py:112
        self._runs = {}

    # ------------------------------------------------------------------------------------------
    def _run(self, B: int) -> _EvalRun:
        r = self._runs.get(B)
        if r is None:
            r = self._runs[B] = _EvalRun(self, B)
        return r

    def _refresh(self):
        """Refresh the eval pack; drop graphs if the parameters were re-homed."""
        eng, P = self.model._engine_and_params()
        if any(P[k].data_ptr() != v.data_ptr() for k, v in self.P.items()):
            self.P = P
            for r in self._runs.values():
                r.graph = None
        eng.repack(self.P, False, _s(), key=self.model._eval_pack_key(self.P))

    def _shortcut_row(self):
        nf = self.model.n_feat
        conv = nn.Conv2d(1, nf, kernel_size=1, stride=1, padding=0)       # diffusion_utilities.py:54
        return torch.cat([conv.weight.detach().reshape(nf), conv.bias.detach()])

    # ------------------------------------------------------------------------------------------
    @torch.no_grad()
    def batch_nll(self, x, c=None) -> torch.Tensor:
        """sum_t mse_t / (2 b_t) per sample (device tensor [B]) — one batch of calculate_likelihood."""
        self._refresh()
        T, B = self.T, x.shape[0]
        r = self._run(B)
        r.load(x, c)
        rows = torch.empty(T, r.row)
        host = self.noise_source == "host"
        if host:
            zs = torch.empty(T, B * r.HW)
        for t in range(1, T + 1):                       # reference order: noise_t, then the model's shortcut
            if host:
                zs[T - t] = torch.randn(x.shape).reshape(-1)
            rows[T - t] = self._shortcut_row()
        r.sc_table.copy_(rows)
        if host:
            r.noise.copy_(zs)
        if self.use_graph and r.graph is None and T >= self.K:
            r.capture(self.K)
            r.acc.zero_()
        r.ctr.fill_(T)
        done = 0
        if r.graph is not None:
            while done + self.K <= T:
                r.graph.replay()
                done += self.K
        s = _s()
        while done < T:
            r.step(s, self.nll_mul, self.nll_div, self.sched.omab)
            done += 1
        return r.acc

    @torch.no_grad()
    def batch_elbo(self, x, c=None) -> torch.Tensor:
        """Per-sample ELBO of code/train_diffusion_paper.py:104-125 (device tensor [B])."""
        self._refresh()
        T, B = self.T, x.shape[0]
        r = self._run(B)
        r.load(x, c)
        host = self.noise_source == "host"
        s = _s()
        for t in torch.linspace(1, T, 10).long():
            ti = int(t)
            if host:
                r.noise[0].copy_(torch.randn(x.shape).reshape(-1))
            r.sc_cur.copy_(self._shortcut_row())
            r.cur_i.fill_(ti)
            r.t_cur.fill_(float(t / T))                # torch.tensor([t / timesteps]) with a tensor t (fp32 divide)
            r._body(s, self.elbo_mul if ti > 1 else None, self.elbo_div, self.sqrt_omab, 0)   # noise row 0
        return r.acc

    def _loop(self, dataloader, fn):
        self.model.eval()                                # the reference leaves the model in eval mode
        total, count = 0.0, 0
        for item in dataloader:
            x, c = _split_batch(item)
            total += fn(x, c).sum().item()
            count += x.shape[0]
        return total, count

    def likelihood(self, dataloader) -> float:
        total, count = self._loop(dataloader, self.batch_nll)
        return total / count

    def elbo_and_bpd(self, dataloader):
        total, count = self._loop(dataloader, self.batch_elbo)
        avg = total / count
        return avg, avg / (64 * 64 * math.log(2))


def _sched_tensors(timesteps, ab_t, b_t, a_t):
    """The caller's schedule as (b_t, a_t, ab_t) fp32 host tensors, or None for the default one.  The reference
    reads ab_t (and b_t) exactly as passed (code/train_diffusion_elbo.py:130,140; code/train_diffusion_paper.py:
    111,122); a missing a_t (unused by both estimators) is derived as 1 - b_t."""
    if ab_t is None and b_t is None and a_t is None:
        return None
    if ab_t is None or b_t is None:
        raise ValueError("pass ab_t and b_t (the tensors the estimators read) or none of the schedule tensors")
    b = torch.as_tensor(b_t).detach().to("cpu", torch.float32).reshape(-1)
    a = (1 - b) if a_t is None else torch.as_tensor(a_t).detach().to("cpu", torch.float32).reshape(-1)
    ab = torch.as_tensor(ab_t).detach().to("cpu", torch.float32).reshape(-1)
    # the reference only indexes [t] for t <= timesteps, so a longer schedule (e.g. built for a larger T) works there
    # too: its first timesteps + 1 entries are the ones read
    n = int(timesteps) + 1
    if min(b.numel(), a.numel(), ab.numel()) < n:
        raise ValueError(f"schedule tensors need at least timesteps + 1 = {n} entries")
    return b[:n].contiguous(), a[:n].contiguous(), ab[:n].contiguous()


def _evaluator(model, timesteps, noise_source="device", sched=None) -> LikelihoodEvaluator:
    cache = model.__dict__.setdefault("_cdm_lik_eval", {})
    skey = None if sched is None else tuple(v.numpy().tobytes() for v in sched)
    key = (int(timesteps), noise_source, skey)
    ev = cache.get(key)
    if ev is None:
        ev = cache[key] = LikelihoodEvaluator(model, timesteps, noise_source, sched_tensors=sched)
    return ev


def calculate_likelihood(model, dataloader, timesteps, device=None, ab_t=None, b_t=None, a_t=None,
                         noise_source: str = "device") -> float:
    """code/train_diffusion_elbo.py:108-149 — mean negative log likelihood (the reference's approximation), under
    the caller's schedule ab_t / b_t when given."""
    sched = _sched_tensors(timesteps, ab_t, b_t, a_t)
    return _evaluator(model, timesteps, noise_source, sched).likelihood(dataloader)


def calculate_elbo_and_bpd_batch(x, pred_noise, noise, t, b_t, a_t, ab_t, dims):
    """code/train_diffusion_elbo.py:74-105 — (elbo, bpd) device scalars for one batch, per-sample t."""
    pred_noise = pred_noise.contiguous(); noise = noise.contiguous()
    B = pred_noise.shape[0]
    HW = pred_noise[0].numel()
    dev = pred_noise.device
    ab = ab_t.to(dev, torch.float32)
    w = (0.5 * (1.0 / (1.0 - ab) - 1.0)).contiguous()
    one = torch.ones_like(w)
    ti = torch.as_tensor(t, device=dev).reshape(-1).to(torch.int32).contiguous()
    acc = torch.zeros(B, device=dev)
    lib().cdm_mse_accum(_p(pred_noise), _p(noise), 0, ab.numel() - 1, B, HW, _p(ti), None, _p(w), _p(one), _p(acc),
                        _s())
    elbo = acc.mean()
    return elbo, elbo / (dims * math.log(2))


def calculate_elbo_and_bpd_dataset(model, dataloader, timesteps, device=None, ab_t=None, b_t=None, a_t=None,
                                   noise_source: str = "device"):
    """code/train_diffusion_paper.py:77-139 — (avg_elbo, bpd) over a dataset, under the caller's schedule when
    given."""
    sched = _sched_tensors(timesteps, ab_t, b_t, a_t)
    return _evaluator(model, timesteps, noise_source, sched).elbo_and_bpd(dataloader)


def calculate_elbo_and_bpd(*args, **kwargs):
    """Both reference signatures: (model, dataloader, timesteps, device, ab_t, b_t, a_t) from
    code/train_diffusion_paper.py:77 and (x, pred_noise, noise, t, b_t, a_t, ab_t, dims) from
    code/train_diffusion_elbo.py:74."""
    first = args[0] if args else kwargs.get("model", kwargs.get("x"))
    if torch.is_tensor(first):
        return calculate_elbo_and_bpd_batch(*args, **kwargs)
    return calculate_elbo_and_bpd_dataset(*args, **kwargs)
