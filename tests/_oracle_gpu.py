"""The CPU oracle's train step (oracle/ref_cpu.py, the functional restatement of the reference) evaluated in fp64 on the
GPU with torch's float64 ops — TEST INFRASTRUCTURE: the checker of the bench-shape tests.  At B = 256, n_feat = 128 an
fp64 train step takes minutes on the box host's CPUs and about a second here; fp64 is the truth both HIP and the
reference's fp32 path are measured against, so where it is computed does not matter (its own error is ~1e-15)."""
import torch
import torch.nn.functional as F

from oracle import ref_cpu as R


def train_step(sd, x, c, noise, t, sc, *, n_feat, n_cfeat=6, height=64, T=1500, lr=1e-5, dtype=torch.float64,
               device="cuda"):
    """perturb_input -> ContextUnet (train BN, the given 1x1 shortcut sc = [w (n_feat) | b (n_feat)]) -> mse ->
    backward -> torch.optim.Adam step (code/train_diffusion_condition.py:216-229).
    Returns (loss, pred, grads, state_dict after the step) on the host."""
    dev = torch.device(device)
    s = {k: (v.to(dtype) if v.is_floating_point() else v.clone()).to(dev) for k, v in sd.items()}
    keys = [k for k, _, kind in R.state_dict_layout(1, n_feat, n_cfeat, height) if kind == "param"]
    for k in keys:
        s[k].requires_grad_(True)
    opt = torch.optim.Adam([s[k] for k in keys], lr=lr)
    _, _, ab = R.make_schedule(T)
    w = sc[:n_feat].reshape(n_feat, 1, 1, 1).to(dtype).to(dev)
    b = sc[n_feat:].to(dtype).to(dev)
    tt = t.to(dev)
    nz = noise.to(dtype).to(dev)
    xp = R.perturb_input(x.to(dtype).to(dev), tt, nz, ab.to(dtype).to(dev))
    pred = R.unet_forward(s, xp, tt / T, c.to(dtype).to(dev), n_feat=n_feat, n_cfeat=n_cfeat, height=height,
                          train=True, shortcut=(w, b))
    loss = F.mse_loss(pred, nz)
    loss.backward()
    grads = {k: s[k].grad.detach().cpu() for k in keys}
    opt.step()
    out = (float(loss), pred.detach().cpu(), grads, {k: v.detach().cpu() for k, v in s.items()})
    del s, opt, pred, loss, xp
    torch.cuda.empty_cache()
    return out
