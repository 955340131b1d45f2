"""ReLU / MaxPool decisions of the piecewise-linear ContextUnet, shared by the gradient parity tests (test-only).

Kinks captures the CPU oracle's decisions (oracle/ref_cpu.py's torch.nn.functional calls, in call order) or imposes
given ones, so that an fp64 autograd run follows the same branch as the run it is compared with; hip_kinks reads HIP's
decisions from one engine forward (the kernels of the module call; deterministic)."""
import torch

from oracle import ref_cpu as R


class Kinks:
    """The oracle's ReLU / MaxPool decisions (torch.nn.functional calls of oracle/ref_cpu.py's forward, in call order):
    capture=True records them (relu: mask z > 0 and z; max_pool2d(2): the first-max index of each 2x2 window, the
    order of torch's CPU kernel); otherwise the given decisions are imposed — relu(z) = z * mask, the pool output taken
    at the given index — so autograd runs the backward of THAT branch of the piecewise-linear network."""

    def __init__(self, relu=None, pool=None):
        self.capture = relu is None
        self.relu, self.pool = ([], []) if self.capture else (list(relu), list(pool))

    def __enter__(self):
        self._relu, self._pool = R.F.relu, R.F.max_pool2d
        it_r, it_p = iter(self.relu), iter(self.pool)

        def relu(z, inplace=False):
            if self.capture:
                self.relu.append(((z > 0).detach().clone(), z.detach().clone()))
                return self._relu(z)
            return z * next(it_r)[0].to(z.dtype)

        def pool(v, k, *a, **kw):
            B, C, H, W = v.shape
            win = v.reshape(B, C, H // 2, 2, W // 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(B, C, H // 2, W // 2, 4)
            if self.capture:
                self.pool.append(first_max(win.detach()))
                return self._pool(v, k, *a, **kw)
            return win.gather(-1, next(it_p).unsqueeze(-1)).squeeze(-1)
        R.F.relu, R.F.max_pool2d = relu, pool
        return self

    def __exit__(self, *exc):
        R.F.relu, R.F.max_pool2d = self._relu, self._pool


def first_max(win):
    """index of the first maximum over the last axis (NaN wins, as torch's CPU max_pool2d and the HIP pool apply)"""
    best = win[..., 0].clone()
    arg = torch.zeros(best.shape, dtype=torch.int64)
    for e in range(1, win.shape[-1]):
        v = win[..., e]
        take = (v > best) | torch.isnan(v)
        best = torch.where(take, v, best)
        arg = torch.where(take, torch.full_like(arg, e), arg)
    return arg


def hip_kinks(m, x, t, c, sc, frozen):
    """HIP's decisions in the oracle's call order, from one engine forward on the same inputs (deterministic, the
    kernels of the module call): per ReLU the mask of z = fma(y, s, t) > 0 (NCHW) and z, per MaxPool the first-max index
    of relu(z) over each window (the pool apply's order).  Call order: the 10 encoder Conv-BN-ReLU layers (a pool after
    the 6th and the 10th), up0's GroupNorm-ReLU, the 8 decoder layers, out.1's GroupNorm-ReLU."""
    eng, P = m._engine_and_params(image_channels_ok=True)
    NF, H, B = m.n_feat, m.h, x.shape[0]
    s = torch.cuda.current_stream().cuda_stream
    eng.repack(P, True, s)
    ws = eng.workspace(B, True, frozen=frozen)
    eng.forward(ws, P, m._to_engine(x.cuda().reshape(B, m.in_channels, H, H)), t.cuda(), c.cuda(),
                sc[0].reshape(-1).cuda(), sc[1].cuda(), B, s, frozen=frozen)
    torch.cuda.synchronize()

    def z_of(y, scale, shift, C, S, per_sample):
        y = y.double().cpu().reshape(B, S, S, C)
        sc_ = scale.double().cpu().reshape(B if per_sample else 1, 1, 1, C)
        sh = shift.double().cpu().reshape(B if per_sample else 1, 1, 1, C)
        z = (y * sc_ + sh).float().permute(0, 3, 1, 2).contiguous()
        return z

    relu, pool = [], []
    L = eng.layers
    for i, l in enumerate(L):
        st = ws.bn[l.name]
        z = z_of(ws.y[l.name], st["scale"], st["shift"], l.cout, l.S, False)
        relu.append((z > 0, z))
        if l.name in ("down1.model.1.conv2", "down2.model.1.conv2"):
            Bz, C, S, _ = z.shape
            r = torch.relu(z)
            win = r.reshape(Bz, C, S // 2, 2, S // 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(Bz, C, S // 2, S // 2, 4)
            pool.append(first_max(win))
        if i == 9:
            z0 = z_of(ws.y0, ws.gn0["scale"], ws.gn0["shift"], 2 * NF, H // 4, True)
            relu.append((z0 > 0, z0))
    zO = z_of(ws.yO, ws.gnO["scale"], ws.gnO["shift"], NF, H, True)
    relu.append((zO > 0, zO))
    return relu, pool


