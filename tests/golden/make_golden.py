"""Generate golden vectors from the REFERENCE itself (build container only; needs /root/reference).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

What it does (and why each piece is legitimate test data, not copied source):
  * imports the reference's ``ContextUnet.py`` + ``code/diffusion_utilities.py`` with an in-memory
    ``torchvision`` stub (torchvision is absent here and none of its symbols is on the hot path:
    diffusion_utilities.py:4,8 import save_image/make_grid/transforms at module level only);
  * AST-lifts ``perturb_input``, ``denoise_add_noise``, ``sample_ddpm``, ``sample_ddpm_from_noise``
    (and ``calculate_likelihood`` / ``calculate_elbo_and_bpd`` from the elbo and paper scripts)
    out of ``code/train_diffusion_condition.py`` (that script runs training at import time, so it
    cannot be imported) and executes them in a namespace that supplies the globals they read;
  * runs them on seeded synthetic inputs (trained weights / CAMELS maps are Git-LFS stubs, F9)
    and writes inputs + outputs as ``.npz`` next to this script.

Nothing from the reference is written to the repo except these numeric outputs.  The reference
directory gains no ``__pycache__`` (bytecode writing is disabled before the import).
"""
from __future__ import annotations

import ast
import json
import os
import sys
import types

sys.dont_write_bytecode = True
REF = os.environ.get("CDM_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))


def _stub_torchvision():
    tv = types.ModuleType("torchvision")
    tvu = types.ModuleType("torchvision.utils")
    tvt = types.ModuleType("torchvision.transforms")
    tvu.save_image = lambda *a, **k: None
    tvu.make_grid = lambda *a, **k: None
    tvt.Compose = lambda *a, **k: None
    tvt.Lambda = lambda *a, **k: None
    tv.utils, tv.transforms = tvu, tvt
    sys.modules.update({"torchvision": tv, "torchvision.utils": tvu, "torchvision.transforms": tvt})


def _lift(path, names, namespace):
    """Compile only the named top-level functions of a reference script into ``namespace``."""
    with open(path) as f:
        tree = ast.parse(f.read(), filename=path)
    defs = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in names]
    missing = set(names) - {d.name for d in defs}
    if missing:
        raise RuntimeError(f"could not lift {missing} from {path}")
    mod = ast.Module(body=defs, type_ignores=[])
    exec(compile(mod, path, "exec"), namespace)
    return namespace


def main():
    _stub_torchvision()
    sys.path[:0] = [os.path.join(REF, "code"), REF]
    import numpy as np
    import torch
    import torch.nn.functional as F
    from ContextUnet import ContextUnet  # noqa: E402  (reference)

    torch.set_num_threads(8)
    T_SAMPLE = 10

    def sched(T, device="cpu"):
        # the reference computes these as script globals (train_diffusion_condition.py:96-99);
        # we evaluate the same expression here to feed the lifted functions.
        beta1, beta2 = 1e-4, 0.02
        b_t = (beta2 - beta1) * torch.linspace(0, 1, T + 1, device=device) + beta1
        a_t = 1 - b_t
        ab_t = torch.cumsum(a_t.log(), dim=0).exp()
        ab_t[0] = 1
        return b_t, a_t, ab_t

    cond_script = os.path.join(REF, "code", "train_diffusion_condition.py")
    lifted_names = ["perturb_input", "denoise_add_noise", "sample_ddpm", "sample_ddpm_from_noise"]

    def sd_np(model):
        return {k: v.detach().cpu().numpy().copy() for k, v in model.state_dict().items()}

    def shortcut_from_seed(seed, nf):
        torch.manual_seed(seed)
        conv = torch.nn.Conv2d(1, nf, kernel_size=1)
        return conv.weight.detach().numpy().copy(), conv.bias.detach().numpy().copy()

    # ---------------- schedules (a1) ----------------
    sc = {}
    for T in (1000, 1500, 2000):
        b, a, ab = sched(T)
        sc[f"b_t_{T}"], sc[f"a_t_{T}"], sc[f"ab_t_{T}"] = b.numpy(), a.numpy(), ab.numpy()
    np.savez(os.path.join(OUT, "schedule.npz"), **sc)

    # ---------------- model fixtures ----------------
    for nf, ncf, B in ((8, 6, 3), (16, 6, 2)):
        torch.manual_seed(0)
        model = ContextUnet(1, nf, ncf, 64)
        fx = {"sd." + k: v for k, v in sd_np(model).items()}
        g = torch.Generator().manual_seed(1234)
        x = torch.rand(B, 1, 64, 64, generator=g)
        t = torch.rand(B, generator=g)
        c = torch.rand(B, ncf, generator=g)
        fx.update(x=x.numpy(), t=t.numpy(), c=c.numpy())

        # eval-mode forward, conditional, per-sample t
        model.eval()
        with torch.no_grad():
            torch.manual_seed(11)
            fx["eval_eps"] = model(x, t, c).numpy()
            fx["eval_sc_w"], fx["eval_sc_b"] = shortcut_from_seed(11, nf)
            # unconditional, t of shape [1,1,1,1] (train_diffusion.py:186) -> broadcast embedding
            t1 = torch.tensor([0.37])[:, None, None, None]
            torch.manual_seed(12)
            fx["eval_uncond_eps"] = model(x, t1, None).numpy()
            fx["eval_uncond_sc_w"], fx["eval_uncond_sc_b"] = shortcut_from_seed(12, nf)
        fx["t1"] = np.array([0.37], dtype=np.float32)

        # train-mode: two steps of the reference train loop body (train_diffusion_condition.py:216-230)
        T = 1500
        b_t, a_t, ab_t = sched(T)
        ns = {"torch": torch, "np": np, "ab_t": ab_t, "a_t": a_t, "b_t": b_t}
        _lift(cond_script, lifted_names, ns)
        model.train()
        optim = torch.optim.Adam(model.parameters(), lr=1e-3)
        for step in range(2):
            torch.manual_seed(100 + step)
            optim.zero_grad()
            noise = torch.randn_like(x)
            tt = torch.randint(1, T + 1, (B,))
            x_pert = ns["perturb_input"](x, tt, noise)
            pred = model(x_pert, tt / T, c)
            loss = F.mse_loss(pred, noise)
            loss.backward()
            if step == 0:
                fx["train0_noise"], fx["train0_t"] = noise.numpy(), tt.numpy()
                fx["train0_xpert"] = x_pert.detach().numpy()
                fx["train0_eps"] = pred.detach().numpy()
                fx["train0_loss"] = np.array(loss.item(), dtype=np.float32)
                for k, p in model.named_parameters():
                    fx["train0_grad." + k] = p.grad.detach().numpy().copy()
            optim.step()
        fx.update({"after2." + k: v for k, v in sd_np(model).items()})
        fx["train_T"] = np.array(T)
        if nf != 8:  # keep the larger model forward-only (grads/Adam are pinned at nf=8)
            fx = {k: v for k, v in fx.items() if not k.startswith(("train0_grad.", "after2."))}
        np.savez_compressed(os.path.join(OUT, f"model_nf{nf}.npz"), **fx)
        print(f"model_nf{nf}: {len(fx)} arrays")

    # ---------------- samplers (a10/a11), CPU RNG order, T=10 ----------------
    nf, ncf = 8, 6
    torch.manual_seed(0)
    model = ContextUnet(1, nf, ncf, 64)
    model.eval()
    ref_sd = np.load(os.path.join(OUT, "model_nf8.npz"))
    for k, v in sd_np(model).items():  # same seed/config as model_nf8.npz: weights are not re-stored
        assert np.array_equal(ref_sd["sd." + k], v), k
    fx = {}
    b_t, a_t, ab_t = sched(T_SAMPLE)
    ns = {"torch": torch, "np": np, "nn_model": model, "b_t": b_t, "a_t": a_t, "ab_t": ab_t,
          "timesteps": T_SAMPLE, "n_cfeat": ncf, "device": torch.device("cpu")}
    _lift(cond_script, lifted_names, ns)
    params = torch.rand(2, ncf, generator=torch.Generator().manual_seed(77))
    fx["params"] = params.numpy()
    for w in (0.0, 1.0, 3.0):
        torch.manual_seed(500)
        xs, inter = ns["sample_ddpm"](n_sample=2, size=64, device=torch.device("cpu"),
                                      params=params, guide_w=w)
        fx[f"sample_w{w:g}"] = xs.numpy()
        fx[f"sample_w{w:g}_inter"] = inter
    # params=None path: random params from the CPU RNG after x_T
    torch.manual_seed(501)
    xs, _ = ns["sample_ddpm"](n_sample=2, size=64, device=torch.device("cpu"), params=None, guide_w=0.0)
    fx["sample_noparams"] = xs.numpy()
    # from-noise reconstruction (:392-399): perturb to T, then reverse
    x0 = torch.rand(2, 1, 64, 64, generator=torch.Generator().manual_seed(78))
    torch.manual_seed(502)
    noise = torch.randn_like(x0)
    xT = ns["perturb_input"](x0, T_SAMPLE, noise)
    xs, inter = ns["sample_ddpm_from_noise"](xT, params, guide_w=1.0)
    fx.update(fromnoise_x0=x0.numpy(), fromnoise_noise=noise.numpy(), fromnoise_xT=xT.numpy(),
              fromnoise_out=xs.numpy(), fromnoise_inter=inter)
    fx["T"] = np.array(T_SAMPLE)
    np.savez_compressed(os.path.join(OUT, "sampler_nf8.npz"), **fx)

    # ---------------- likelihood / ELBO estimators (next-1), CPU RNG order ----------------
    # calculate_likelihood (code/train_diffusion_elbo.py:108-149), calculate_elbo_and_bpd dataset form
    # (code/train_diffusion_paper.py:77-139) and per-batch form (code/train_diffusion_elbo.py:74-105)
    elbo_script = os.path.join(REF, "code", "train_diffusion_elbo.py")
    paper_script = os.path.join(REF, "code", "train_diffusion_paper.py")
    fx = {}
    gl = torch.Generator().manual_seed(90)
    batches = [(torch.rand(2, 1, 64, 64, generator=gl), torch.rand(2, ncf, generator=gl)),
               (torch.rand(1, 1, 64, 64, generator=gl), torch.rand(1, ncf, generator=gl))]  # ragged last batch
    for j, (xb, pb) in enumerate(batches):
        fx[f"lik_x{j}"], fx[f"lik_c{j}"] = xb.numpy(), pb.numpy()
    ns_e = {"torch": torch, "np": np, "F": F}
    _lift(elbo_script, ["calculate_likelihood", "calculate_elbo_and_bpd"], ns_e)
    ns_p = {"torch": torch, "np": np, "F": F}
    _lift(paper_script, ["calculate_likelihood", "calculate_elbo_and_bpd"], ns_p)
    T_LIK = 10
    b_t, a_t, ab_t = sched(T_LIK)
    torch.manual_seed(600)
    fx["nll_elbo_script"] = np.array(ns_e["calculate_likelihood"](model, batches, T_LIK, "cpu", ab_t, b_t, a_t))
    torch.manual_seed(600)
    fx["nll_paper_script"] = np.array(ns_p["calculate_likelihood"](model, batches, T_LIK, "cpu", ab_t, b_t, a_t))
    T_ELBO = 1500
    b_t, a_t, ab_t = sched(T_ELBO)
    torch.manual_seed(601)
    elbo, bpd = ns_p["calculate_elbo_and_bpd"](model, batches, T_ELBO, "cpu", ab_t, b_t, a_t)
    fx["paper_elbo"], fx["paper_bpd"] = np.array(elbo), np.array(bpd)
    # per-batch form on a (x, pred_noise, noise, t) quadruple
    ge = torch.Generator().manual_seed(91)
    xq = torch.rand(5, 1, 64, 64, generator=ge); pq = torch.randn(5, 1, 64, 64, generator=ge)
    nq = torch.randn(5, 1, 64, 64, generator=ge); tq = torch.randint(1, T_ELBO + 1, (5,), generator=ge)
    e, bp = ns_e["calculate_elbo_and_bpd"](xq, pq, nq, tq, b_t, a_t, ab_t, 64 * 64)
    fx.update(batch_x=xq.numpy(), batch_pred=pq.numpy(), batch_noise=nq.numpy(), batch_t=tq.numpy(),
              batch_elbo=e.numpy(), batch_bpd=bp.numpy())
    fx["T_lik"], fx["T_elbo"] = np.array(T_LIK), np.array(T_ELBO)
    np.savez_compressed(os.path.join(OUT, "likelihood_nf8.npz"), **fx)
    print("likelihood:", {k: float(v) for k, v in fx.items() if v.ndim == 0})

    # ---------------- layout metadata at the bench config ----------------
    torch.manual_seed(0)
    m = ContextUnet(1, 128, 6, 64)
    meta = {"keys": [[k, list(v.shape), str(v.dtype)] for k, v in m.state_dict().items()],
            "n_params": sum(p.numel() for p in m.parameters())}
    with open(os.path.join(OUT, "layout_nf128.json"), "w") as f:
        json.dump(meta, f)
    print("done")


if __name__ == "__main__":
    main()
