#!/usr/bin/env python3
"""train_diffusion.py — drop-in CLI of the reference, on the MI355X HIP engine.

    python camels-diffusion-model_amd/train_diffusion.py LR EPOCHS TIMESTEPS [NUM_PARAMS] [--options]
    torchrun --nproc-per-node N camels-diffusion-model_amd/train_diffusion.py ...      (data parallel)

Positional arguments keep the reference semantics:
  3 args  (code/train_diffusion.py:74-76)   unconditional training, n_cfeat = 5, c = None,
          outputs/BIGnoiselr_{lr}_epochs_{E}_timesteps_{T}/, checkpoints model_epoch_{ep}.pth at ep+1 in
          {25, 50, 75, 100}; afterwards the reconstruct-from-noised sampler (:163-193).
  4 args  (README.md:68-73 / code/train_diffusion_condition.py:74-77) parameter-conditioned training,
          n_cfeat = NUM_PARAMS, outputs/paper_lr_{lr}_epochs_{E}_timesteps_{T}_params_{P}/, validation MSE
          every 5 epochs, checkpoints model_epoch_{ep+1}.pth every 25 epochs and at the end; then CFG sampling
          and conditioned reconstruction of held-out maps.
Per epoch the learning rate is lr*(1 - ep/E) (:213); batch size 32, n_feat 128, 64x64 (:82-85).
Data parallel (torchrun, N ranks): --batch-size is per rank, each step is one global batch of N x batch-size
samples of the epoch's permutation split across the ranks (trainer.shard_epoch), and an epoch whose loss turned
NaN / inf stops the run (device-side counter, one read per epoch).

Data (code/train_diffusion_condition.py:104-160): Maps_HI_IllustrisTNG_LH_z=0.00.npy [N,256,256] -> shift
to positive, /max, log10, min-max to [0,1], bilinear to 64x64; params.npy [N/15, 6] repeated x15, per-column
min-max (param_min/max.npy saved), first NUM_PARAMS columns; 1500 held out with random_split(seed 42).
The CAMELS files are not in this repository (Git-LFS stubs upstream): pass --data/--params, or --synthetic N
to train on synthetic maps of the same shape.
Plots of the reference (loss curves, PDFs, P(k)) are analysis, outside the hot path: losses, samples and
timings are written as .npy / .log instead.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cdm_amd.data import preprocess_maps, preprocess_params, train_test_split  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("lr", type=float)
    ap.add_argument("epochs", type=int)
    ap.add_argument("timesteps", type=int)
    ap.add_argument("num_params", type=int, nargs="?", default=None)
    ap.add_argument("--data", default="../data/Maps_HI_IllustrisTNG_LH_z=0.00.npy")
    ap.add_argument("--params", default="../data/params.npy")
    ap.add_argument("--synthetic", type=int, default=0, help="train on N synthetic maps (no CAMELS files needed)")
    ap.add_argument("--batch-size", type=int, default=32)
    ap.add_argument("--n-feat", type=int, default=128)
    ap.add_argument("--height", type=int, default=64)
    ap.add_argument("--out-root", default="outputs")
    ap.add_argument("--n-samples", type=int, default=10)
    ap.add_argument("--guide-w", type=float, default=0.0)
    ap.add_argument("--no-sample", action="store_true")
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args(argv)

    world = int(os.environ.get("WORLD_SIZE", "1")); rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    import cdm_amd
    from cdm_amd import DDPM, ContextUnet, Trainer
    from cdm_amd.trainer import shard_epoch

    conditional = a.num_params is not None
    n_cfeat = a.num_params if conditional else 5
    if conditional:
        out_dir = os.path.join(a.out_root, f"paper_lr_{a.lr}_epochs_{a.epochs}_timesteps_{a.timesteps}_params_{a.num_params}")
    else:
        out_dir = os.path.join(a.out_root, f"BIGnoiselr_{a.lr}_epochs_{a.epochs}_timesteps_{a.timesteps}")
    save_dir = os.path.join(out_dir, "weights")
    if rank == 0:
        os.makedirs(save_dir, exist_ok=True)
    H = a.height

    # ------------------------------- data -------------------------------
    if a.synthetic:
        g = torch.Generator().manual_seed(1234)
        n = a.synthetic - a.synthetic % 15 if a.synthetic >= 15 else a.synthetic
        maps = torch.rand(n, 1, H, H, generator=g)
        raw_params = torch.rand(max(1, n // 15), 6, generator=g).numpy().astype(np.float64)
        params = preprocess_params(raw_params, n, n_cfeat) if n % 15 == 0 else torch.rand(n, n_cfeat, generator=g)
    else:
        torch.cuda.set_device(local)
        maps = preprocess_maps(np.load(a.data, mmap_mode="r"), H)          # device pipeline (csrc/data.hip)
        params = preprocess_params(np.load(a.params), maps.shape[0], n_cfeat, out_dir if rank == 0 else None) \
            if conditional else torch.zeros(maps.shape[0], n_cfeat)
    n_total = maps.shape[0]
    if conditional:
        # random_split(full, [n - 1500, 1500], seed 42) (:150-156); small synthetic sets hold out 10 %
        train_idx, test_idx = train_test_split(n_total, min(1500, n_total // 10), 42)
    else:
        train_idx, test_idx = torch.arange(n_total), torch.arange(0)
    # data-parallel sharding: every rank sees a disjoint slice of each epoch's permutation
    dev = torch.device("cuda", local)
    maps_d, params_d = maps.to(dev), params.to(dev)
    if rank == 0:
        with open(os.path.join(out_dir, "dataset_info.txt"), "w") as f:
            f.write(f"Total dataset size: {n_total}\nTrain dataset size: {len(train_idx)}\n"
                    f"Test dataset size: {len(test_idx)}\nNumber of parameters used for conditioning: {n_cfeat}\n"
                    f"World size: {world}\n")

    # ------------------------------- model / trainer -------------------------------
    torch.manual_seed(a.seed)
    model = ContextUnet(1, a.n_feat, n_cfeat, H).to(dev)
    trainer = Trainer(model, a.lr, a.timesteps, a.batch_size, seed=a.seed)
    log = open(os.path.join(out_dir, "timing_and_performance.log"), "a") if rank == 0 else None
    loss_log, val_log = [], []
    t_train0 = time.time()
    for ep in range(a.epochs):
        t_ep = time.time()
        lr = a.lr * (1 - ep / a.epochs)
        trainer.set_lr(lr)
        model.train()
        order = train_idx[torch.randperm(len(train_idx), generator=torch.Generator().manual_seed(a.seed * 7919 + ep))]
        ep_loss, nb = torch.zeros(1, device=dev), 0
        # every rank runs the same number of steps; ragged global batches are weighted by sample count
        for idx, count in shard_epoch(order, a.batch_size, world, rank):
            idx = idx.to(dev)
            loss = trainer.step(maps_d[idx], params_d[idx] if conditional else None,
                                global_count=count if world > 1 and count != a.batch_size * world else None)
            ep_loss += loss
            nb += 1
        bad = trainer.check_finite()                 # SURVEY §5 failure guard: one host read per epoch
        if bad:
            raise FloatingPointError(f"epoch {ep + 1}: {bad} training step(s) produced a NaN / inf loss "
                                     f"(lr {lr:.3e}); stopping before the checkpoint is overwritten")
        torch.cuda.synchronize()
        ep_time = time.time() - t_ep
        loss_log.append(float(ep_loss.item()) / max(nb, 1))
        msg = f"Epoch {ep + 1}/{a.epochs}, Train Loss: {loss_log[-1]:.6f}, lr {lr:.3e}, epoch time {ep_time:.2f}s"
        if conditional and (ep % 5 == 0 or ep == a.epochs - 1) and len(test_idx):
            val_log.append(validation_mse(model, maps_d[test_idx.to(dev)], params_d[test_idx.to(dev)], trainer.sched,
                                          a.timesteps, a.batch_size))
            msg += f", Val Loss: {val_log[-1]:.6f}"
        if rank == 0:
            print(msg, flush=True)
            log.write(msg + "\n"); log.flush()
            save_now = ((ep + 1) % 25 == 0 or ep == a.epochs - 1) if conditional else (ep + 1) in (25, 50, 75, 100)
            if save_now:
                name = f"model_epoch_{ep + 1}.pth" if conditional else f"model_epoch_{ep}.pth"
                torch.save({k: v.detach().cpu() for k, v in model.state_dict().items()}, os.path.join(save_dir, name))
    total_train = time.time() - t_train0
    if rank == 0:
        np.save(os.path.join(out_dir, "loss_log.npy"), np.array(loss_log))
        if val_log:
            np.save(os.path.join(out_dir, "val_loss_log.npy"), np.array(val_log))
        log.write(f"Total training time: {total_train:.2f} s\n")

    # ------------------------------- sampling -------------------------------
    if not a.no_sample and rank == 0:
        model.eval()
        d = DDPM(model, a.timesteps, dev)
        ns = a.n_samples
        src = test_idx if len(test_idx) else torch.arange(min(ns, n_total))
        sel = src[:ns].to(dev)
        x = maps_d[sel]
        p = params_d[sel] if conditional else None
        noise = torch.randn(x.shape, device=dev)
        x_T = cdm_amd.perturb_input(x, a.timesteps, noise, d.sched)
        t0 = time.time()
        rec, inter = d.sample_ddpm_from_noise(x_T, p, guide_w=a.guide_w)
        torch.cuda.synchronize()
        dt = time.time() - t0
        np.save(os.path.join(out_dir, "reconstructed_images.npy"), rec.cpu().numpy())
        np.save(os.path.join(out_dir, "intermediate.npy"), inter)
        log.write(f"Reconstruction of {ns} maps, T={a.timesteps}: {dt:.2f} s\n")
        # the reference's post-sampling statistics (code/train_diffusion.py:250, diffusion_utilities.py:370),
        # on the HIP statistics kernels; the plotted arrays go to .npz files
        cdm_amd.compare_distributions(x[:, 0].cpu().numpy(), rec[:, 0].cpu().numpy(), out_dir)
        cdm_amd.compare_power_spectra(x, rec, out_dir)
        if conditional:
            t0 = time.time()
            samples, _ = d.sample_ddpm(ns, H, dev, p, a.guide_w)
            torch.cuda.synchronize()
            dt = time.time() - t0
            np.save(os.path.join(out_dir, "generated_samples.npy"), samples.cpu().numpy())
            log.write(f"Sampling {ns} maps (w={a.guide_w}), T={a.timesteps}: {dt:.2f} s ({ns / dt:.3f} img/s)\n")
        with open(os.path.join(out_dir, "means.txt"), "w") as f:
            f.write(f"Processed Images Mean: {x.mean().item()}\nReconstructed Images Mean: {rec.mean().item()}\n")
    if log:
        log.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    return out_dir


@torch.no_grad()
def validation_mse(model, x, c, sched, T, bs):
    """Validation pass (code/train_diffusion_condition.py:235-251): eval mode, fresh noise / t, mean MSE."""
    import cdm_amd
    model.eval()
    tot, n = 0.0, 0
    for i in range(0, x.shape[0], bs):
        xb, cb = x[i:i + bs], c[i:i + bs]
        noise = torch.randn_like(xb)
        t = torch.randint(1, T + 1, (xb.shape[0],), device=xb.device)
        xp = cdm_amd.perturb_input(xb, t, noise, sched)
        pred = model(xp, t.float() / T, cb)
        tot += F.mse_loss(pred, noise).item()
        n += 1
    model.train()
    return tot / max(n, 1)


if __name__ == "__main__":
    main()
