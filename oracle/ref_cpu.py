"""CPU oracle for the ContextUnet DDPM hot path — TEST INFRASTRUCTURE ONLY.

This module is the checker, never the product: only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import it.  The shipped path (``cdm_amd``) runs on the HIP
library and fails loudly when it is missing; nothing in it routes through this file.

It is a *functional* restatement (plain ``torch.nn.functional`` on CPU, fp32) of the reference
algorithm, operating on a reference-layout ``state_dict`` (same 156 keys, OIHW weights).  It is
pinned against golden vectors produced by the reference itself (``tests/golden/make_golden.py``,
run in the build container where ``/root/reference`` exists); ``tests/test_oracle_golden.py``
checks it bit-for-bit on CPU.

Reference citations (paths relative to the reference repo root):
  schedule            code/train_diffusion_condition.py:87-88,96-99 (== code/train_diffusion.py:85-86,94-97)
  perturb_input       code/train_diffusion_condition.py:202-203   (non-standard (1-ab) noise factor)
  denoise_add_noise   code/train_diffusion_condition.py:274-279
  sample_ddpm (CFG)   code/train_diffusion_condition.py:281-335; functional form code/sample_power_spectra.py:71-110
  sample_from_noise   code/train_diffusion_condition.py:337-384
  ContextUnet.forward ContextUnet.py:42-60 (== code/train_diffusion.py:48-66)
  ResidualConvBlock   code/diffusion_utilities.py:13-65 (random 1x1 shortcut :50-55)
  UnetUp / UnetDown   code/diffusion_utilities.py:79-116
  EmbedFC             code/diffusion_utilities.py:118-145
  train step          code/train_diffusion_condition.py:206-232 (Adam :200, LR decay :213)
  likelihood (NLL)    code/train_diffusion_elbo.py:108-149 (== code/train_diffusion_paper.py:142-183)
  ELBO/BPD, dataset   code/train_diffusion_paper.py:77-139
  ELBO/BPD, per batch code/train_diffusion_elbo.py:74-105
"""
from __future__ import annotations

import math
from typing import Callable, Dict, List, Optional, Tuple

import torch
import torch.nn.functional as F

BN_EPS = 1e-5
BN_MOMENTUM = 0.1
GN_EPS = 1e-5
BETA1, BETA2 = 1e-4, 0.02


# ----------------------------------------------------------------------------------------------
# a1: schedule
# ----------------------------------------------------------------------------------------------
def make_schedule(timesteps: int, beta1: float = BETA1, beta2: float = BETA2):
    """b_t, a_t, ab_t as fp32 CPU vectors of length T+1 (code/train_diffusion_condition.py:96-99).

    ab_t is exp(cumsum(log a_t)) — not cumprod — and ab_t[0] is forced to 1.
    """
    b_t = (beta2 - beta1) * torch.linspace(0, 1, timesteps + 1) + beta1
    a_t = 1 - b_t
    ab_t = torch.cumsum(a_t.log(), dim=0).exp()
    ab_t[0] = 1
    return b_t, a_t, ab_t


# ----------------------------------------------------------------------------------------------
# a2 / a9: elementwise diffusion math
# ----------------------------------------------------------------------------------------------
def perturb_input(x, t, noise, ab_t):
    """sqrt(ab[t])*x + (1-ab[t])*noise   (code/train_diffusion_condition.py:202-203)."""
    return ab_t.sqrt()[t, None, None, None] * x + (1 - ab_t[t, None, None, None]) * noise


def denoise_add_noise(x, t, pred_noise, z, b_t, a_t, ab_t):
    """(x - eps*(1-a)/sqrt(1-ab))/sqrt(a) + sqrt(b)*z   (code/train_diffusion_condition.py:274-279)."""
    if z is None:
        z = torch.randn_like(x)
    noise = b_t.sqrt()[t] * z
    mean = (x - pred_noise * ((1 - a_t[t]) / (1 - ab_t[t]).sqrt())) / a_t[t].sqrt()
    return mean + noise


# ----------------------------------------------------------------------------------------------
# a3..a7: the denoiser, functional over a reference-layout state_dict
# ----------------------------------------------------------------------------------------------
def draw_shortcut(in_ch: int, out_ch: int, generator_device: str = "cpu"):
    """The reference builds a *fresh* nn.Conv2d(in,out,1) on every forward (diffusion_utilities.py:54).

    Constructing one here consumes the CPU RNG exactly as the reference does (weight via
    kaiming_uniform_(a=sqrt(5)), then bias), so a seeded oracle replays the same draws.
    """
    conv = torch.nn.Conv2d(in_ch, out_ch, kernel_size=1, stride=1, padding=0)
    return conv.weight.detach().clone(), conv.bias.detach().clone()


class _Ctx:
    def __init__(self, sd: Dict[str, torch.Tensor], train: bool):
        self.sd = sd
        self.train = train

    def bn(self, x, name):
        sd = self.sd
        out = F.batch_norm(x, sd[name + ".running_mean"], sd[name + ".running_var"],
                           sd[name + ".weight"], sd[name + ".bias"], training=self.train,
                           momentum=BN_MOMENTUM, eps=BN_EPS)
        if self.train:
            nbt = sd[name + ".num_batches_tracked"]
            nbt.add_(1)
        return out

    def conv_bn_relu(self, x, name):
        # name + ".0" conv3x3 p1, name + ".1" BatchNorm2d, ReLU   (diffusion_utilities.py:26-37)
        y = F.conv2d(x, self.sd[name + ".0.weight"], self.sd[name + ".0.bias"], stride=1, padding=1)
        return F.relu(self.bn(y, name + ".1"))

    def res_block(self, x, name, is_res=False, shortcut=None):
        x1 = self.conv_bn_relu(x, name + ".conv1")
        x2 = self.conv_bn_relu(x1, name + ".conv2")
        if not is_res:
            return x2
        if x.shape[1] == x2.shape[1]:
            return x + x2
        w, b = shortcut() if callable(shortcut) else shortcut
        return F.conv2d(x, w, b) + x2

    def embed(self, v, name, in_dim):
        v = v.reshape(-1, in_dim).to(self.sd[name + ".model.0.weight"].dtype)
        h = F.linear(v, self.sd[name + ".model.0.weight"], self.sd[name + ".model.0.bias"])
        h = F.gelu(h)
        return F.linear(h, self.sd[name + ".model.2.weight"], self.sd[name + ".model.2.bias"])

    def down(self, x, name):
        x = self.res_block(x, name + ".model.0")
        x = self.res_block(x, name + ".model.1")
        return F.max_pool2d(x, 2)

    def up(self, x, skip, name):
        x = torch.cat((x, skip), 1)
        x = F.conv_transpose2d(x, self.sd[name + ".model.0.weight"], self.sd[name + ".model.0.bias"],
                               stride=2)
        x = self.res_block(x, name + ".model.1")
        return self.res_block(x, name + ".model.2")


def unet_forward(sd: Dict[str, torch.Tensor], x: torch.Tensor, t: torch.Tensor,
                 c: Optional[torch.Tensor], *, n_feat: int, n_cfeat: int, height: int,
                 train: bool, shortcut) -> torch.Tensor:
    """ContextUnet.forward (ContextUnet.py:42-60) on CPU fp32.

    ``shortcut`` is either a (w, b) pair or a zero-arg callable drawing one (the reference draws
    it from the CPU RNG inside the forward).  In train mode BN running stats in ``sd`` are updated
    in place, as nn.BatchNorm2d does.
    """
    ctx = _Ctx(sd, train)
    h = height
    x0 = ctx.res_block(x, "init_conv", is_res=True, shortcut=shortcut)
    d1 = ctx.down(x0, "down1")
    d2 = ctx.down(d1, "down2")
    hv = F.gelu(F.avg_pool2d(d2, h // 4))
    if c is None:
        c = torch.zeros(x0.shape[0], n_cfeat).to(x0)
    cemb1 = ctx.embed(c, "contextembed1", n_cfeat).view(-1, 2 * n_feat, 1, 1)
    temb1 = ctx.embed(t, "timeembed1", 1).view(-1, 2 * n_feat, 1, 1)
    cemb2 = ctx.embed(c, "contextembed2", n_cfeat).view(-1, n_feat, 1, 1)
    temb2 = ctx.embed(t, "timeembed2", 1).view(-1, n_feat, 1, 1)
    u1 = F.conv_transpose2d(hv, sd["up0.0.weight"], sd["up0.0.bias"], stride=h // 4)
    u1 = F.relu(F.group_norm(u1, 8, sd["up0.1.weight"], sd["up0.1.bias"], eps=GN_EPS))
    u2 = ctx.up(cemb1 * u1 + temb1, d2, "up1")
    u3 = ctx.up(cemb2 * u2 + temb2, d1, "up2")
    o = torch.cat((u3, x0), 1)
    o = F.conv2d(o, sd["out.0.weight"], sd["out.0.bias"], padding=1)
    o = F.relu(F.group_norm(o, 8, sd["out.1.weight"], sd["out.1.bias"], eps=GN_EPS))
    return F.conv2d(o, sd["out.3.weight"], sd["out.3.bias"], padding=1)


# ----------------------------------------------------------------------------------------------
# reference parameter layout (names/shapes of the 156-entry state_dict)
# ----------------------------------------------------------------------------------------------
def state_dict_layout(in_channels: int, n_feat: int, n_cfeat: int, height: int):
    """Ordered list of (key, shape, kind) of the reference state_dict (ContextUnet.py:13-40)."""
    nf = n_feat
    out: List[Tuple[str, tuple, str]] = []

    def conv(name, cin, cout, k):
        out.append((name + ".weight", (cout, cin, k, k), "param"))
        out.append((name + ".bias", (cout,), "param"))

    def bn(name, ch):
        out.append((name + ".weight", (ch,), "param"))
        out.append((name + ".bias", (ch,), "param"))
        out.append((name + ".running_mean", (ch,), "buffer"))
        out.append((name + ".running_var", (ch,), "buffer"))
        out.append((name + ".num_batches_tracked", (), "buffer"))

    def rcb(name, cin, cout):
        conv(name + ".conv1.0", cin, cout, 3); bn(name + ".conv1.1", cout)
        conv(name + ".conv2.0", cout, cout, 3); bn(name + ".conv2.1", cout)

    def lin(name, i, o):
        out.append((name + ".weight", (o, i), "param"))
        out.append((name + ".bias", (o,), "param"))

    def convt(name, cin, cout, k):
        out.append((name + ".weight", (cin, cout, k, k), "param"))
        out.append((name + ".bias", (cout,), "param"))

    rcb("init_conv", in_channels, nf)
    rcb("down1.model.0", nf, nf); rcb("down1.model.1", nf, nf)
    rcb("down2.model.0", nf, 2 * nf); rcb("down2.model.1", 2 * nf, 2 * nf)
    for name, i, o in (("timeembed1", 1, 2 * nf), ("timeembed2", 1, nf),
                       ("contextembed1", n_cfeat, 2 * nf), ("contextembed2", n_cfeat, nf)):
        lin(name + ".model.0", i, o); lin(name + ".model.2", o, o)
    convt("up0.0", 2 * nf, 2 * nf, height // 4)
    out.append(("up0.1.weight", (2 * nf,), "param")); out.append(("up0.1.bias", (2 * nf,), "param"))
    convt("up1.model.0", 4 * nf, nf, 2); rcb("up1.model.1", nf, nf); rcb("up1.model.2", nf, nf)
    convt("up2.model.0", 2 * nf, nf, 2); rcb("up2.model.1", nf, nf); rcb("up2.model.2", nf, nf)
    conv("out.0", 2 * nf, nf, 3)
    out.append(("out.1.weight", (nf,), "param")); out.append(("out.1.bias", (nf,), "param"))
    conv("out.3", nf, in_channels, 3)
    return out


def clone_sd(sd):
    return {k: v.detach().cpu().clone() for k, v in sd.items()}


# ----------------------------------------------------------------------------------------------
# a8: one training step (perturb -> forward(train) -> mse -> backward -> Adam)
# ----------------------------------------------------------------------------------------------
class OracleTrainer:
    """Stateful CPU train step matching code/train_diffusion_condition.py:206-232.

    Parameters live in ``self.sd`` (leaf tensors with grad), Adam is ``torch.optim.Adam`` with
    the reference defaults; ``lr`` is set per call (the reference sets it per epoch, :213).
    """

    def __init__(self, sd, *, n_feat, n_cfeat, height, in_channels=1, lr=1e-5):
        self.cfg = dict(n_feat=n_feat, n_cfeat=n_cfeat, height=height)
        layout = state_dict_layout(in_channels, n_feat, n_cfeat, height)
        self.param_keys = [k for k, _, kind in layout if kind == "param"]
        self.sd = clone_sd(sd)
        for k in self.param_keys:
            self.sd[k].requires_grad_(True)
        self.opt = torch.optim.Adam([self.sd[k] for k in self.param_keys], lr=lr)

    def step(self, x0, c, noise, t_int, timesteps, ab_t, shortcut, lr=None):
        if lr is not None:
            self.opt.param_groups[0]["lr"] = lr
        self.opt.zero_grad()
        x_pert = perturb_input(x0, t_int, noise, ab_t)
        pred = unet_forward(self.sd, x_pert, t_int / timesteps, c, train=True, shortcut=shortcut,
                            **self.cfg)
        loss = F.mse_loss(pred, noise)
        loss.backward()
        grads = {k: self.sd[k].grad.detach().clone() for k in self.param_keys}
        self.opt.step()
        return loss.detach(), pred.detach(), grads


def adam_step_restated(p, g, m, v, lr, step, beta1=0.9, beta2=0.999, eps=1e-8, grad_scale=1.0):
    """One torch.optim.Adam step (torch/optim/adam.py _single_tensor_adam, the reference's optimizer,
    code/train_diffusion_condition.py:200,229) restated elementwise in numpy fp32 with the roundings of torch's
    CPU kernels: lerp_ = fma(w, g - m, m); mul_(b2).addcmul_ = fma((1-b2) g, g, v b2); denom = sqrt(v) / bc2s + eps;
    addcdiv_ = p + (-step_size * m) / denom; step_size / bc2s from Python-float bias corrections, cast to fp32.
    sqrt is correctly rounded here (torch's vectorised CPU sqrt may differ by an ulp, host-dependently).  fma is
    evaluated as an exact fp64 product plus an fp64 add, then rounded (a double rounding can differ from a true
    fma on ~1e-9 of the inputs).  Returns (p, m, v) as new float32 arrays."""
    import numpy as np
    f32 = np.float32

    def fma(a, b, c):
        return (np.float64(a) * np.asarray(b, np.float64) + np.asarray(c, np.float64)).astype(f32)
    gi = (np.asarray(g, f32) * f32(grad_scale)).astype(f32)
    bc1 = 1 - beta1 ** float(step)
    bc2s = f32((1 - beta2 ** float(step)) ** 0.5)
    nss = f32(-(lr / bc1))
    m = fma(f32(1 - beta1), (gi - m).astype(f32), m)
    v = fma((f32(1 - beta2) * gi).astype(f32), gi, (np.asarray(v, f32) * f32(beta2)).astype(f32))
    denom = (np.sqrt(v) / bc2s + f32(eps)).astype(f32)
    return (np.asarray(p, f32) + ((nss * m).astype(f32) / denom).astype(f32)).astype(f32), m, v


# ----------------------------------------------------------------------------------------------
# a10 / a11: samplers (CFG), replaying the reference RNG order on the CPU generator
# ----------------------------------------------------------------------------------------------
def _snap(i, timesteps, save_rate):
    return i % save_rate == 0 or i == timesteps or i < 8


def sample_loop(model: Callable, x: torch.Tensor, params, guide_w: float, timesteps: int, sched,
                save_rate: int = 20, noise_fn: Optional[Callable] = None):
    """The shared T..1 loop of sample_ddpm / sample_ddpm_from_noise (:312-333 / :361-382).

    ``model(x, t, c)`` is called once (w == 0) or twice (cond first, then uncond with c = 0).
    ``noise_fn(i, x)`` returns z for step i (default: torch.randn_like, the CPU-path RNG order).
    """
    b_t, a_t, ab_t = sched
    uncond = torch.zeros_like(params) if params is not None else None
    inter = []
    for i in range(timesteps, 0, -1):
        t = torch.tensor([i / timesteps])
        if i > 1:
            z = noise_fn(i, x) if noise_fn is not None else torch.randn_like(x)
        else:
            z = 0
        if guide_w > 0 and params is not None:
            ec = model(x, t, params)
            eu = model(x, t, uncond)
            eps = eu + guide_w * (ec - eu)
        else:
            eps = model(x, t, params)
        x = denoise_add_noise(x, i, eps, z, b_t, a_t, ab_t)
        if _snap(i, timesteps, save_rate):
            inter.append(x.detach().clone())
    return x, torch.stack(inter) if inter else None


def sample_ddpm(model, n_sample, size, params, guide_w, timesteps, sched, n_cfeat, save_rate=20):
    """code/train_diffusion_condition.py:281-335: x_T ~ randn (CPU RNG), params ~ rand if None."""
    x = torch.randn(n_sample, 1, size, size)
    if params is None:
        params = torch.rand(n_sample, n_cfeat)
    return sample_loop(model, x, params, guide_w, timesteps, sched, save_rate)


def sample_ddpm_from_noise(model, noise_images, params, guide_w, timesteps, sched, save_rate=20):
    """code/train_diffusion_condition.py:337-384 (start from a given tensor)."""
    return sample_loop(model, noise_images.clone(), params, guide_w, timesteps, sched, save_rate)


def make_model_fn(sd, *, n_feat, n_cfeat, height, train=False, shortcut_log=None):
    """model(x, t, c) closure drawing a fresh shortcut per call from the CPU RNG (F5)."""
    def draw():
        w, b = draw_shortcut(1, n_feat)
        if shortcut_log is not None:
            shortcut_log.append((w, b))
        return w, b

    def fn(x, t, c):
        with torch.no_grad():
            return unet_forward(sd, x, t, c, n_feat=n_feat, n_cfeat=n_cfeat, height=height,
                                train=train, shortcut=draw)
    return fn


# ----------------------------------------------------------------------------------------------
# next-1: likelihood / ELBO estimators (model(x, t, c) as from make_model_fn, eval mode)
def calculate_likelihood(model: Callable, batches, timesteps: int, sched) -> float:
    """code/train_diffusion_elbo.py:108-149: sum_t mse_t / (2 b_t) per sample, t = 1..T ascending,
    x_t = sqrt(ab) x + (1 - ab) noise (same non-standard factor as perturb_input); noise ~ randn_like
    (CPU RNG, drawn before the model call, whose shortcut draw follows)."""
    b_t, a_t, ab_t = sched
    total, count = 0.0, 0
    for x, param in batches:
        bsz = x.shape[0]
        acc = torch.zeros(bsz)
        for t in range(1, timesteps + 1):
            noise = torch.randn_like(x)
            x_t = ab_t.sqrt()[t, None, None, None] * x + (1 - ab_t[t, None, None, None]) * noise
            pred = model(x_t, torch.tensor([t / timesteps]), param)
            mse = F.mse_loss(pred, noise, reduction="none").mean(dim=[1, 2, 3])
            acc += mse / (2 * b_t[t])
        total += acc.sum().item()
        count += bsz
    return total / count


def calculate_elbo_and_bpd_dataset(model: Callable, batches, timesteps: int, sched):
    """code/train_diffusion_paper.py:77-139: 10 evenly spaced t (linspace(1,T,10).long()), standard
    sqrt(1 - ab) noise factor, weight 0.5 b/(1 - ab) for t > 1, /10; bpd over 64*64 dims."""
    b_t, a_t, ab_t = sched
    total, count = 0.0, 0
    for x, param in batches:
        bsz = x.shape[0]
        acc = torch.zeros(bsz)
        for t in torch.linspace(1, timesteps, 10).long():
            noise = torch.randn_like(x)
            x_t = ab_t.sqrt()[t] * x + torch.sqrt(1 - ab_t[t]) * noise
            pred = model(x_t, torch.tensor([t / timesteps]), param)
            mse = F.mse_loss(pred, noise, reduction="none").mean(dim=[1, 2, 3])
            if t > 1:
                w = 0.5 * (b_t[t] / (1.0 - ab_t[t]))
                acc += w * mse / 10.0
        total += acc.sum().item()
        count += bsz
    avg = total / count
    return avg, avg / (64 * 64 * math.log(2))


def calculate_elbo_and_bpd_batch(x, pred_noise, noise, t, b_t, a_t, ab_t, dims):
    """code/train_diffusion_elbo.py:74-105 (per training batch, per-sample t)."""
    mse = F.mse_loss(pred_noise, noise, reduction="none").mean(dim=[1, 2, 3])
    w = 0.5 * (1.0 / (1.0 - ab_t[t]) - 1.0)
    elbo = (w * mse).mean()
    return elbo, elbo / (dims * math.log(2))


def forward_flops(n_feat: int, height: int, in_channels: int = 1, n_cfeat: int = 6) -> float:
    """Algorithmic forward FLOPs per image (2 per MAC) — SURVEY §8(d) basis (19.178788 GF @ nf=128)."""
    nf, H = n_feat, height
    f = 0.0
    conv = lambda cin, cout, hw: 2.0 * cin * cout * 9 * hw * hw
    f += conv(in_channels, nf, H) + conv(nf, nf, H)                    # init_conv
    f += in_channels * nf * H * H * 2.0                                 # random 1x1 shortcut
    f += 4 * conv(nf, nf, H)                                            # down1
    f += conv(nf, 2 * nf, H // 2) + 3 * conv(2 * nf, 2 * nf, H // 2)    # down2
    f += 2.0 * (4 * nf) * nf * 4 * (H // 4) ** 2                        # up1 convT 2x2
    f += 4 * conv(nf, nf, H // 2)
    f += 2.0 * (2 * nf) * nf * 4 * (H // 2) ** 2                        # up2 convT 2x2
    f += 4 * conv(nf, nf, H)
    f += 2.0 * (2 * nf) * (2 * nf) * (H // 4) ** 2                      # up0 convT k=H/4 from 1x1
    f += conv(2 * nf, nf, H) + conv(nf, in_channels, H)                 # out
    f += 2.0 * ((1 + n_cfeat) * 3 * nf + 2 * (4 * nf * nf + nf * nf))  # EmbedFC x4
    return f
