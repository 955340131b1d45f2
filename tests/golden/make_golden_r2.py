"""Round-2 golden vectors from the REFERENCE itself (build container only; needs /root/reference).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_r2.py

Same mechanism as make_golden.py (the reference's ContextUnet.py + code/diffusion_utilities.py imported with an
in-memory torchvision stub; perturb_input / sample_ddpm AST-lifted from code/train_diffusion_condition.py), for
the two things round 1 left unpinned:

  train_nf8.npz    three iterations of the reference training loop body (train_diffusion_condition.py:213-229):
                   optim.param_groups[0]['lr'] = lrate*(1-ep/n_epoch) per epoch (:213), zero_grad, randn_like
                   noise, randint t, perturb_input, forward (train BN, fresh CPU-RNG 1x1 shortcut), mse, backward,
                   Adam step (:200).  Steps 0 and 1 run at epoch 0 (lr = 1e-3), step 2 at epoch 1 of 4 (lr =
                   7.5e-4), so the LR decay path is exercised.  Stored per step: the draws (noise, t, shortcut w/b)
                   so the HIP trainer can replay them, the loss, and the full state_dict after the step.
  sampler_T1500_nf8.npz
                   sample_ddpm (:281-335) at the benchmarked T = 1500 with the CPU RNG order of the reference's CPU
                   run, n = 2, w in {0, 3}: x_T seed, final x, and a subset of the 82 snapshots (indices listed).
                   Also the same trajectories re-run by the CPU oracle in fp64 (oracle/ref_cpu.py, fed the same
                   draws), whose distance to the fp32 reference is the accuracy the reference's own fp32 path has
                   at T = 1500 (the tolerance basis of tests/test_gpu_trainer_sampler_r2.py).

Nothing from the reference is written to the repo except these numeric outputs.
"""
from __future__ import annotations

import os
import sys
import time

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from make_golden import REF, _lift, _stub_torchvision  # noqa: E402

OUT = HERE
SNAP_KEEP = (0, 1, 5, 25, 50, 74, 75, 76, 77, 78, 79, 80, 81)   # of the 82 snapshots at T=1500, save_rate=20


def main():
    _stub_torchvision()
    sys.path[:0] = [os.path.join(REF, "code"), REF]
    import numpy as np
    import torch
    import torch.nn.functional as F
    from ContextUnet import ContextUnet  # noqa: E402  (reference)

    torch.set_num_threads(8)
    cond_script = os.path.join(REF, "code", "train_diffusion_condition.py")
    lifted = ["perturb_input", "denoise_add_noise", "sample_ddpm", "sample_ddpm_from_noise"]

    def sched(T):
        beta1, beta2 = 1e-4, 0.02
        b_t = (beta2 - beta1) * torch.linspace(0, 1, T + 1) + beta1
        a_t = 1 - b_t
        ab_t = torch.cumsum(a_t.log(), dim=0).exp()
        ab_t[0] = 1
        return b_t, a_t, ab_t

    def sd_np(model):
        return {k: v.detach().cpu().numpy().copy() for k, v in model.state_dict().items()}

    base = np.load(os.path.join(OUT, "model_nf8.npz"))

    # ---------------- training loop body, 3 iterations ----------------
    nf, ncf, T, lrate, n_epoch = 8, 6, 1500, 1e-3, 4
    torch.manual_seed(0)
    model = ContextUnet(1, nf, ncf, 64)
    for k, v in sd_np(model).items():
        assert np.array_equal(base["sd." + k], v), k           # same seeded weights as model_nf8.npz
    x = torch.from_numpy(base["x"].copy()); c = torch.from_numpy(base["c"].copy())
    B = x.shape[0]
    b_t, a_t, ab_t = sched(T)
    ns = {"torch": torch, "np": np, "ab_t": ab_t, "a_t": a_t, "b_t": b_t}
    _lift(cond_script, lifted, ns)
    model.train()
    optim = torch.optim.Adam(model.parameters(), lr=lrate)
    fx = {"x": x.numpy(), "c": c.numpy(), "T": np.array(T), "lrate": np.array(lrate), "n_epoch": np.array(n_epoch)}
    for step, ep in enumerate((0, 0, 1)):
        optim.param_groups[0]["lr"] = lrate * (1 - ep / n_epoch)
        torch.manual_seed(200 + step)
        optim.zero_grad()
        noise = torch.randn_like(x)
        tt = torch.randint(1, T + 1, (B,))
        st = torch.get_rng_state()
        conv = torch.nn.Conv2d(1, nf, kernel_size=1)          # record the draw the forward is about to make
        fx[f"s{step}_sc_w"] = conv.weight.detach().numpy().reshape(nf).copy()
        fx[f"s{step}_sc_b"] = conv.bias.detach().numpy().copy()
        torch.set_rng_state(st)
        x_pert = ns["perturb_input"](x, tt, noise)
        pred = model(x_pert, tt / T, c)
        loss = F.mse_loss(pred, noise)
        loss.backward()
        optim.step()
        fx[f"s{step}_noise"], fx[f"s{step}_t"] = noise.numpy(), tt.numpy()
        fx[f"s{step}_lr"] = np.array(optim.param_groups[0]["lr"])
        fx[f"s{step}_loss"] = np.array(loss.item(), dtype=np.float32)
        fx.update({f"s{step}_after.{k}": v for k, v in sd_np(model).items()})
        if step == 0:
            fx.update({"s0_grad." + k: p.grad.detach().numpy().copy() for k, p in model.named_parameters()})
    np.savez_compressed(os.path.join(OUT, "train_nf8.npz"), **fx)
    print("train_nf8:", len(fx), "arrays; losses", [float(fx[f"s{i}_loss"]) for i in range(3)])

    # ---------------- sampler at T = 1500 ----------------
    from oracle import ref_cpu as R
    torch.manual_seed(0)
    model = ContextUnet(1, nf, ncf, 64)
    model.eval()
    Ts = 1500
    b_t, a_t, ab_t = sched(Ts)
    ns = {"torch": torch, "np": np, "nn_model": model, "b_t": b_t, "a_t": a_t, "ab_t": ab_t, "timesteps": Ts,
          "n_cfeat": ncf, "device": torch.device("cpu")}
    _lift(cond_script, lifted, ns)
    params = torch.from_numpy(np.load(os.path.join(OUT, "sampler_nf8.npz"))["params"].copy())
    sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in model.state_dict().items()}
    sched64 = tuple(v.double() for v in sched(Ts))
    fx = {"params": params.numpy(), "T": np.array(Ts), "snap_keep": np.array(SNAP_KEEP)}
    for w, seed in ((0.0, 700), (3.0, 701)):
        t0 = time.time()
        torch.manual_seed(seed)
        xs, inter = ns["sample_ddpm"](n_sample=2, size=64, device=torch.device("cpu"), params=params, guide_w=w)
        assert inter.shape[0] == 82
        fx[f"w{w:g}_seed"] = np.array(seed)
        fx[f"w{w:g}_x"] = xs.numpy()
        fx[f"w{w:g}_inter"] = inter[list(SNAP_KEEP)]
        # fp64 re-run of the same trajectory (same CPU-RNG draws, oracle network in fp64)
        torch.manual_seed(seed)
        x64 = torch.randn(2, 1, 64, 64).double()

        def model64(xx, t, cc):
            wgt, bias = R.draw_shortcut(1, nf)
            with torch.no_grad():
                return R.unet_forward(sd64, xx, t.double(), cc, n_feat=nf, n_cfeat=ncf, height=64, train=False,
                                      shortcut=(wgt.double(), bias.double()))

        x64f, inter64 = R.sample_loop(model64, x64, params.double(), w, Ts, sched64, 20,
                                      noise_fn=lambda i, xx: torch.randn(xx.shape).double())
        fx[f"w{w:g}_x_fp64"] = x64f.numpy()
        fx[f"w{w:g}_inter_fp64"] = inter64.numpy()[list(SNAP_KEEP)]
        mx = np.abs(fx[f"w{w:g}_x_fp64"]).max()
        d = np.abs(fx[f"w{w:g}_x"] - fx[f"w{w:g}_x_fp64"]).max() / mx
        print(f"T=1500 w={w:g}: {time.time() - t0:.1f} s, max|x| {mx:.3g}, fp32 ref vs fp64 max|d|/max|x| {d:.3e}")
    np.savez_compressed(os.path.join(OUT, "sampler_T1500_nf8.npz"), **fx)
    print("done")


if __name__ == "__main__":
    main()
