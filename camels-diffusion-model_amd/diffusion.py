"""DDPM schedule, perturbation, denoising and the T-step (CFG) sampler on the HIP engine.

API mirrors the reference:
  schedule                      code/train_diffusion_condition.py:96-99
  perturb_input(x, t, noise)    :202-203   (non-standard (1 - ab) noise factor)
  denoise_add_noise(...)        :274-279
  sample_ddpm(n, size, device, params, guide_w)            :281-335  -> (x, intermediate)
  sample_ddpm_from_noise(noise_images, params, save_rate, guide_w)   :337-384
  functional sample_ddpm(model, ..., timesteps, b_t, a_t, ab_t)      code/sample_power_spectra.py:71-110
  unconditional reconstruction sampler                    code/train_diffusion.py:170-193

The sampler captures K denoise steps (prologue -> full ContextUnet eval forward -> fused
CFG-combine + denoise + snapshot) in one hipGraph and replays it; a device-side step counter makes
each captured step read its own timestep, coefficients, shortcut draw and noise stream, and the
reference's `intermediate.append(x.cpu())` snapshots are written on device into a preallocated
buffer (copied to host once at the end).

RNG modes (``z_source``):
  "device": z from on-device Philox; x_T / random params / per-forward shortcut draws consume the CPU
            RNG in exactly the order the reference's *GPU* run does (its z come from the CUDA generator).
  "host":   everything from the CPU RNG in the order of the reference's *CPU* run (x_T, then per step
            z then shortcut(s)); z is pre-drawn into a device table — bit-compatible with the oracle.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch
import torch.nn as nn

from ._lib import lib

BETA1, BETA2 = 1e-4, 0.02


def _s():
    return torch.cuda.current_stream().cuda_stream


def _p(t):
    return None if t is None else t.data_ptr()


def sqrt_scalar_f32(v: torch.Tensor) -> torch.Tensor:
    """fp32 sqrt of every element as a 0-d tensor op computes it: IEEE correctly rounded, the same on every host
    (round(sqrt_fp64(x)) equals the correctly rounded fp32 sqrt: 53 >= 2 * 24 + 2 bits)."""
    return torch.from_numpy(np.sqrt(v.detach().cpu().double().numpy()).astype(np.float32))


class Schedule:
    """b_t, a_t, ab_t (T+1) computed with the reference's fp32 expressions on the host, plus the
    per-step coefficient tables the kernels read (same fp32 operations as the reference).

    The reference's denoise_add_noise (code/train_diffusion_condition.py:274-279) takes sqrt in two forms: of the whole
    vector, ``b_t.sqrt()[t]``, and of indexed 0-d scalars, ``a_t[t].sqrt()`` and ``(1 - ab_t[t]).sqrt()``.  torch's
    vectorised CPU sqrt is not correctly rounded and differs between hosts in a few entries (round 5: the MI355X box's
    host and the container that made the golden trajectories disagree in ``sqrt(b_t)``, ``sqrt(a_t)`` and
    ``sqrt(1 - ab_t)``, tools/traj_diag.py, profiles/r5_traj_diag.json), while the 0-d form is IEEE everywhere.  So the
    scalar forms are built with :func:`sqrt_scalar_f32` (host-independent, equal to the reference's values on any host)
    and the vector forms (``sqrt(b_t)`` here, ``sqrt(ab_t)`` of perturb_input, :202-203) with torch's vector sqrt on
    this host, as the reference evaluates them; ``sb`` replaces the latter with a given table (the trajectory parity
    tests pass the golden host's, tests/golden/schedule.npz)."""

    def __init__(self, timesteps: int, device="cuda", beta1: float = BETA1, beta2: float = BETA2, tensors=None,
                 sb: Optional[torch.Tensor] = None):
        """``tensors=(b_t, a_t, ab_t)`` uses a caller's schedule (the functional sampler of
        code/sample_power_spectra.py:71-110 takes them as arguments) instead of building the default one."""
        self.T = int(timesteps)
        if tensors is not None:
            b_t, a_t, ab_t = (torch.as_tensor(v).detach().to("cpu", torch.float32).reshape(-1) for v in tensors)
            if not (b_t.numel() == a_t.numel() == ab_t.numel() == self.T + 1):
                raise ValueError(f"schedule tensors must have timesteps + 1 = {self.T + 1} entries")
        else:
            b_t = (beta2 - beta1) * torch.linspace(0, 1, self.T + 1) + beta1
            a_t = 1 - b_t
            ab_t = torch.cumsum(a_t.log(), dim=0).exp()
            ab_t[0] = 1
        dev = torch.device(device)
        self.b_t, self.a_t, self.ab_t = b_t.to(dev), a_t.to(dev), ab_t.to(dev)
        self.sab = ab_t.sqrt().to(dev)                       # perturb: ab_t.sqrt()[t] (vector form)
        self.omab = (1 - ab_t).to(dev)                       #          (1 - ab[t])
        # denoise: (1 - a_t[t]) / (1 - ab_t[t]).sqrt() and a_t[t].sqrt() (0-d forms), b_t.sqrt()[t] (vector form);
        # fp32 subtraction / division in numpy: IEEE like torch's
        oma = (1 - a_t).numpy()
        with np.errstate(divide="ignore", invalid="ignore"):   # entry 0 (1 - ab_t[0] = 0) is never used: t >= 1
            self.coef = torch.from_numpy((oma / sqrt_scalar_f32(1 - ab_t).numpy()).astype(np.float32)).to(dev)
        self.sa = sqrt_scalar_f32(a_t).to(dev)
        if sb is not None:
            sb = torch.as_tensor(sb).detach().to("cpu", torch.float32).reshape(-1)
            if sb.numel() != self.T + 1:
                raise ValueError(f"sb must have timesteps + 1 = {self.T + 1} entries")
            self.sb = sb.to(dev)
        else:
            self.sb = b_t.sqrt().to(dev)

    def tensors(self):
        return self.b_t, self.a_t, self.ab_t


def _as_i32(t, n, device):
    if isinstance(t, int) or (torch.is_tensor(t) and t.dim() == 0):
        return torch.full((n,), int(t), dtype=torch.int32, device=device)
    t = torch.as_tensor(t, device=device).reshape(-1).to(torch.int32)
    return t.expand(n).contiguous() if t.numel() == 1 else t.contiguous()


def perturb_input(x, t, noise, sched: Schedule):
    """sqrt(ab[t]) x + (1 - ab[t]) noise  (code/train_diffusion_condition.py:202-203); t int or [B]."""
    x = x.contiguous(); noise = noise.contiguous()
    B = x.shape[0]
    out = torch.empty_like(x)
    ti = _as_i32(t, B, x.device)
    lib().cdm_perturb(_p(x), _p(noise), _p(ti), None, 0, _p(sched.sab), _p(sched.omab), B, x[0].numel(), sched.T,
                      _p(out), None, _s())
    return out


def denoise_add_noise(x, t: int, pred_noise, z, sched: Schedule):
    """(x - eps (1-a)/sqrt(1-ab)) / sqrt(a) + sqrt(b) z   (code/train_diffusion_condition.py:274-279)."""
    x = x.contiguous(); pred_noise = pred_noise.contiguous()
    if z is None:
        z = torch.randn_like(x)
    if not torch.is_tensor(z):                      # the reference passes z = 0 at the last step
        z = torch.full_like(x, float(z))
    z = z.contiguous()
    out = torch.empty_like(x)
    cur = torch.full((1,), int(t), dtype=torch.int32, device=x.device)
    T = max(int(t), sched.T)
    # z_table with stride 0: z[e] for every step; force i > 1 semantics by the table itself
    lib().cdm_denoise(_p(x), _p(out), None, x.numel(), _p(pred_noise), 0, 0.0, _p(cur), _p(sched.coef),
                      _p(sched.sa), _p(sched.sb), _p(z), 0, 0, None, None, None, T, _s())
    if int(t) <= 1 and z.abs().max().item() != 0:  # kernel treats i == 1 as z = 0 (reference passes 0 there)
        out = out + sched.b_t.sqrt()[int(t)] * z
    return out


def snapshot_slots(T: int, save_rate: int = 20):
    """slot index per step i (reference: i % save_rate == 0 or i == T or i < 8), in append order."""
    slots = np.full(T + 1, -1, dtype=np.int32)
    k = 0
    for i in range(T, 0, -1):
        if i % save_rate == 0 or i == T or i < 8:
            slots[i] = k
            k += 1
    return slots, k


class GraphSampler:
    """One reverse-diffusion run (T steps) of ContextUnet on the HIP engine, hipGraph-replayed."""

    def __init__(self, model, sched: Schedule, n: int, guide_w: float, params: Optional[torch.Tensor],
                 save_rate: int = 20, z_source: str = "device", steps_per_graph: int = 10, seed: int = 1234,
                 snapshots: bool = True, use_graph: bool = True):
        from .model import ContextUnet  # noqa: F401
        self.model, self.sched, self.n = model, sched, n
        self.T = sched.T
        self.guide_w = float(guide_w)
        self.cfg = self.guide_w > 0 and params is not None
        self.z_source = z_source
        self.seed = seed
        eng, P = model._engine_and_params()
        self.eng, self.P = eng, P
        dev = P["out.3.weight"].device
        self.dev = dev
        H, nf, ncf = model.h, model.n_feat, model.n_cfeat
        self.H = H
        B = 2 * n if self.cfg else n
        self.B = B
        self.sets = 2 if self.cfg else 1
        s = _s()
        eng.repack(P, False, s, key=model._eval_pack_key(P))
        self.ws = eng.workspace(B, False)
        E = lambda *sh: torch.empty(*sh, device=dev)
        self.xbuf = E(B, H, H)
        self.cbuf = torch.zeros(B, ncf, device=dev)
        if params is not None:
            self.cbuf[:n] = params.to(dev, torch.float32).reshape(n, ncf)
        self.has_c = params is not None
        self.t_cur = E(1)
        self.cur_i = torch.zeros(1, dtype=torch.int32, device=dev)
        self.ctr = torch.zeros(1, dtype=torch.int32, device=dev)
        self.row = 2 * self.sets * nf
        self.sc_table = E(self.T, self.row)
        self.sc_cur = E(self.row)
        slots, nslots = snapshot_slots(self.T, save_rate)
        self.nslots = nslots if snapshots else 0
        self.slot = torch.from_numpy(slots).to(dev) if snapshots else None
        self.snaps = E(max(self.nslots, 1), n * H * H)
        self.z_table = E(max(self.T - 1, 1), n * H * H) if z_source == "host" else None
        self.zseed = torch.zeros(1, dtype=torch.int64, device=dev)    # per-run Philox key (device z mode)
        self.K = max(1, int(steps_per_graph))
        self.use_graph = use_graph
        self.graph = None

    # RNG draws in the reference order ------------------------------------------------------------
    def _draw_shortcut_row(self):
        nf = self.model.n_feat
        ws, bs = [], []
        for _ in range(self.sets):
            conv = nn.Conv2d(1, nf, kernel_size=1, stride=1, padding=0)
            ws.append(conv.weight.detach().reshape(nf)); bs.append(conv.bias.detach())
        return torch.cat(ws + bs)

    def prepare_rng(self, host_z: bool):
        """Draw the per-step CPU-RNG quantities (and z in host mode) in reference order."""
        n, H = self.n, self.H
        rows = []
        zs = [] if host_z else None
        for i in range(self.T, 0, -1):
            if host_z and i > 1:
                zs.append(torch.randn(n, 1, H, H))
            rows.append(self._draw_shortcut_row())
        self.sc_table.copy_(torch.stack(rows))
        if host_z and zs:
            self.z_table.copy_(torch.stack(zs).reshape(self.T - 1, n * H * H))

    # one step --------------------------------------------------------------------------------------
    def _step(self, s):
        lb = lib()
        nf, n = self.model.n_feat, self.n
        lb.cdm_sample_prologue(_p(self.ctr), self.T, _p(self.cur_i), _p(self.t_cur), _p(self.sc_table), self.row,
                               _p(self.sc_cur), s)
        half = self.sets * nf
        sc_w, sc_b = self.sc_cur[:half], self.sc_cur[half:]
        eps = self.eng.forward(self.ws, self.P, self.xbuf, self.t_cur, self.cbuf, sc_w, sc_b, n, s)
        numel = n * self.H * self.H
        lb.cdm_denoise(_p(self.xbuf), _p(self.xbuf), _p(self.xbuf) if self.cfg else None, numel, _p(eps),
                       1 if self.cfg else 0, self.guide_w, _p(self.cur_i), _p(self.sched.coef), _p(self.sched.sa),
                       _p(self.sched.sb), _p(self.z_table), numel, self.seed, _p(self.zseed), _p(self.slot),
                       _p(self.snaps), self.T, s)

    def _capture(self):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            # warm-up launch of every kernel before capture (code objects resident)
            self.ctr.fill_(self.T)
            self._step(s.cuda_stream)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(self.K):
                self._step(torch.cuda.current_stream().cuda_stream)
        self.graph = g

    def prepare(self):
        """Refresh the eval weight pack and capture the step graph (idempotent)."""
        eng, P = self.model._engine_and_params()
        if any(P[k].data_ptr() != v.data_ptr() for k, v in self.P.items()):
            self.P, self.graph = P, None                    # parameters were re-homed: re-capture
        eng.repack(self.P, False, _s(), key=self.model._eval_pack_key(self.P))
        if self.use_graph and self.graph is None and self.T >= self.K:
            self._capture()

    def run(self, x_T: torch.Tensor, steps: Optional[int] = None):
        """Run T steps (or the first ``steps``) from x_T [n,1,H,H].

        Returns (x [n,1,H,H], intermediate np [slots,n,1,H,H] or None)."""
        n, H = self.n, self.H
        if self.z_source == "device":
            # fresh z for every run, drawn from torch's CUDA generator (the reference's randn_like(x) on the device
            # consumes it too): reproducible under torch.cuda.manual_seed, different across consecutive calls.
            # Drawn before prepare(): a graph capture moves the generator's offset.
            self.zseed.random_()
        self.prepare()
        total = self.T if steps is None else min(int(steps), self.T)
        self.xbuf[:n] = x_T.to(self.dev, torch.float32).reshape(n, H, H)
        if self.cfg:
            self.xbuf[n:] = self.xbuf[:n]
        self.ctr.fill_(self.T)
        done = 0
        if self.graph is not None:
            while done + self.K <= total:
                self.graph.replay()
                done += self.K
        s = _s()
        while done < total:
            self._step(s)
            done += 1
        x = self.xbuf[:n].reshape(n, 1, H, H).clone()
        inter = None
        if self.nslots:
            inter = self.snaps[: self.nslots].reshape(self.nslots, n, 1, H, H).cpu().numpy()
        return x, inter


class DDPM:
    """Script-globals bundle of the reference (nn_model, timesteps, b_t/a_t/ab_t, n_cfeat, device)."""

    def __init__(self, model, timesteps: int, device="cuda", z_source: str = "device", seed: int = 1234,
                 sched_tensors=None, sched_sb=None):
        """sched_tensors = (b_t, a_t, ab_t) and sched_sb = the b_t.sqrt() table to use (Schedule); None: built here."""
        self.model, self.T = model, int(timesteps)
        self.sched = Schedule(self.T, device, tensors=sched_tensors, sb=sched_sb)
        self.b_t, self.a_t, self.ab_t = self.sched.tensors()
        self.device = torch.device(device)
        self.n_cfeat = model.n_cfeat
        self.z_source = z_source
        self.seed = seed
        self._samplers = {}

    def perturb_input(self, x, t, noise):
        return perturb_input(x, t, noise, self.sched)

    def denoise_add_noise(self, x, t, pred_noise, z=None):
        return denoise_add_noise(x, t, pred_noise, z, self.sched)

    def _sampler(self, n, guide_w, params, save_rate):
        key = (n, float(guide_w) if params is not None else 0.0, params is not None, save_rate, self.z_source)
        smp = self._samplers.get(key)
        if smp is None:
            smp = self._samplers[key] = GraphSampler(self.model, self.sched, n, guide_w, params, save_rate,
                                                     self.z_source, seed=self.seed)
        elif params is not None:
            smp.cbuf[:n] = params.to(smp.dev, torch.float32).reshape(n, -1)
        return smp

    @torch.no_grad()
    def sample_ddpm(self, n_sample=1, size=64, device=None, params=None, guide_w=0.0, save_rate=20):
        """code/train_diffusion_condition.py:281-335 -> (samples, intermediate)."""
        assert size == self.model.h
        host = self.z_source == "host"
        x_T = torch.randn(n_sample, 1, size, size)          # CPU RNG, as the reference
        if params is None:
            params = torch.rand(n_sample, self.n_cfeat)      # CPU RNG, as the reference
        smp = self._sampler(n_sample, guide_w, params, save_rate)
        smp.prepare_rng(host_z=host)
        return smp.run(x_T)

    @torch.no_grad()
    def sample_ddpm_from_noise(self, noise_images, params=None, save_rate=20, guide_w=0.0):
        """code/train_diffusion_condition.py:337-384 (and the unconditional code/train_diffusion.py:170-193)."""
        n = noise_images.shape[0]
        smp = self._sampler(n, guide_w, params, save_rate)
        smp.prepare_rng(host_z=self.z_source == "host")
        return smp.run(noise_images)


@torch.no_grad()
def sample_ddpm(model, n_sample=1, size=64, device=None, params=None, guide_w=0.0, timesteps=1000, b_t=None,
                a_t=None, ab_t=None, z_source="device"):
    """Functional sampler of code/sample_power_spectra.py:71-110 (returns the final x only).  b_t / a_t / ab_t are
    the caller's schedule, as in the reference (all three or none: None builds the default schedule)."""
    given = [v is not None for v in (b_t, a_t, ab_t)]
    if any(given) and not all(given):
        raise ValueError("pass all of b_t, a_t, ab_t or none of them")
    d = DDPM(model, timesteps, device or model.out[3].weight.device, z_source=z_source,
             sched_tensors=(b_t, a_t, ab_t) if all(given) else None)
    if params is None:
        x_T = torch.randn(n_sample, 1, size, size)
        params = torch.rand(n_sample, 6 if model.n_cfeat == 6 else model.n_cfeat)
        smp = d._sampler(n_sample, guide_w, params, 20)
        smp.prepare_rng(host_z=z_source == "host")
        return smp.run(x_T)[0]
    x, _ = d.sample_ddpm(n_sample, size, device, params, guide_w)
    return x
