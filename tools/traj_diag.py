"""Trajectory input audit (VERDICT r4 "next" 1): which input of the n_feat = 128, T = 400 golden trajectory differs on the
GPU box from the container that made the golden (tests/golden/make_golden_r4.py)?

    python tools/traj_diag.py record        # build container: writes tools/traj_diag_container.npz
    python tools/traj_diag.py compare       # GPU box: the same run there (CPU oracle + HIP), first differing quantity

Per step of the first NSTEPS reverse steps (w = 0, seed 800, the reference's CPU-RNG order: x_T, then per step z and the
shortcut draw) this records a SHA-256 of every input the trajectory consumes — the seeded weights, the schedule and the
coefficient tables derived from it on the host, params, x_T, each z, each shortcut (w, b), t — and the CPU oracle's eps
and x after the step (full arrays).  `compare` recomputes all of it on the box, prints the first quantity whose hash
differs, and where eps / x differ, by how much; it also steps the HIP sampler one step at a time on the box's draws and
reports its distance to both.  Test infrastructure (imports oracle/), never on the product path.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from oracle import ref_cpu as R  # noqa: E402
import _parity  # noqa: E402

NSTEPS = 21
OUT = os.path.join(ROOT, "tools", "traj_diag_container.npz")


def _h(t) -> str:
    a = t.detach().cpu().numpy() if torch.is_tensor(t) else np.asarray(t)
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:20]


def run_cpu(nsteps: int = NSTEPS, threads: int = 8):
    import cdm_amd
    torch.set_num_threads(threads)
    sfx = np.load(os.path.join(ROOT, "tests", "golden", "sampler_T400_nf128.npz"))
    T, nf = int(sfx["T"]), int(sfx["n_feat"])
    rec, arr = {}, {}
    torch.manual_seed(int(sfx["init_seed"]))
    m = cdm_amd.ContextUnet(1, nf, 6, 64)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    hs = hashlib.sha256()
    for k in sorted(sd):
        hs.update(k.encode()); hs.update(np.ascontiguousarray(sd[k].numpy()).tobytes())
        rec["sd:" + k] = _h(sd[k])
    rec["sd"] = hs.hexdigest()[:20]
    b_t, a_t, ab_t = _parity.golden_schedule(T)
    rec.update({"b_t": _h(b_t), "a_t": _h(a_t), "ab_t": _h(ab_t)})
    # the tables the HIP sampler derives on the host (diffusion.Schedule), same expressions
    rec["coef"] = _h((1 - a_t) / (1 - ab_t).sqrt()); rec["sa"] = _h(a_t.sqrt()); rec["sb"] = _h(b_t.sqrt())
    params = torch.from_numpy(sfx["params"])
    rec["params"] = _h(params)
    seed = int(sfx["w0_seed"])
    torch.manual_seed(seed)
    x = torch.randn(2, 1, 64, 64)
    rec["x_T"] = _h(x)
    arr["x_T"] = x.numpy().copy()
    draws = {"z": [], "sc_w": [], "sc_b": []}
    for k, i in enumerate(range(T, T - nsteps, -1)):
        t = torch.tensor([i / T])
        z = torch.randn_like(x)
        w, b = R.draw_shortcut(1, nf)
        draws["z"].append(z); draws["sc_w"].append(w.reshape(-1)); draws["sc_b"].append(b)
        with torch.no_grad():
            eps = R.unet_forward(sd, x, t, params, n_feat=nf, n_cfeat=6, height=64, train=False, shortcut=(w, b))
        x = R.denoise_add_noise(x, i, eps, z, b_t, a_t, ab_t)
        for name, v in (("t", t), ("z", z), ("sc_w", w), ("sc_b", b), ("eps", eps), ("x", x)):
            rec[f"{name}_{k}"] = _h(v)
        arr[f"eps_{k}"] = eps.numpy().copy(); arr[f"x_{k}"] = x.numpy().copy()
    gold = sfx["w0_inter"][1]                       # the golden's snapshot after step 380 (= NSTEPS steps)
    rec["x_after_21_equals_golden_snapshot1"] = bool(np.array_equal(x.numpy(), gold)) if nsteps == 21 else None
    rec["x_after_21_dev_vs_golden_fp64"] = float(np.abs(x.numpy().astype(np.float64) - sfx["w0_inter_fp64"][1]).max()
                                                 / np.abs(sfx["w0_inter_fp64"][1]).max()) if nsteps == 21 else None
    rec["cpu_capability"] = torch.backends.cpu.get_cpu_capability()
    rec["torch_threads"] = torch.get_num_threads()
    rec["torch"] = torch.__version__
    return rec, arr, (sd, params, seed, T, nf, draws, (b_t, a_t, ab_t))


def run_hip(ctx, nsteps: int = NSTEPS):
    """The HIP sampler (eval engine, host z table) stepped one step at a time on the same draws: eps and x per step."""
    import cdm_amd
    from cdm_amd.diffusion import GraphSampler, Schedule
    sd, params, seed, T, nf, draws, sched = ctx
    m = cdm_amd.ContextUnet(1, nf, 6, 64)
    m.load_state_dict(sd)
    m = m.cuda().eval()
    sch = Schedule(T, "cuda", tensors=sched)
    smp = GraphSampler(m, sch, 2, 0.0, params, z_source="host", use_graph=False)
    torch.manual_seed(seed)
    x_T = torch.randn(2, 1, 64, 64)
    smp.prepare_rng(host_z=True)                 # same CPU order as the oracle run: z, shortcut per step
    eps_l, x_l = [], []
    smp.prepare()
    n, H = 2, 64
    smp.xbuf[:n] = x_T.cuda().reshape(n, H, H)
    smp.ctr.fill_(T)
    from cdm_amd._lib import lib
    s = torch.cuda.current_stream().cuda_stream
    for k in range(nsteps):
        lb = lib()
        lb.cdm_sample_prologue(smp.ctr.data_ptr(), T, smp.cur_i.data_ptr(), smp.t_cur.data_ptr(), smp.sc_table.data_ptr(),
                               smp.row, smp.sc_cur.data_ptr(), s)
        half = nf
        eps = smp.eng.forward(smp.ws, smp.P, smp.xbuf, smp.t_cur, smp.cbuf, smp.sc_cur[:half], smp.sc_cur[half:], n, s)
        eps_l.append(eps.detach().cpu().numpy().reshape(n, 1, H, H).copy())
        numel = n * H * H
        lb.cdm_denoise(smp.xbuf.data_ptr(), smp.xbuf.data_ptr(), None, numel, eps.data_ptr(), 0, 0.0, smp.cur_i.data_ptr(),
                       sch.coef.data_ptr(), sch.sa.data_ptr(), sch.sb.data_ptr(), smp.z_table.data_ptr(), numel, smp.seed,
                       smp.zseed.data_ptr(), smp.slot.data_ptr(), smp.snaps.data_ptr(), T, s)
        x_l.append(smp.xbuf[:n].detach().cpu().numpy().reshape(n, 1, H, H).copy())
    zt = smp.z_table[:nsteps].detach().cpu()
    zsame = all(torch.equal(zt[k], draws["z"][k].reshape(-1)) for k in range(nsteps))
    scsame = all(torch.equal(smp.sc_table[k, :nf].cpu(), draws["sc_w"][k]) and
                 torch.equal(smp.sc_table[k, nf:].cpu(), draws["sc_b"][k]) for k in range(nsteps))
    return eps_l, x_l, {"hip_z_table_equals_oracle_draws": zsame, "hip_shortcut_table_equals_oracle_draws": scsame}


def _dev(a, b):
    a = np.asarray(a, np.float64); b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "record"
    if mode == "record":
        rec, arr, _ = run_cpu()
        np.savez_compressed(OUT, rec=np.array(json.dumps(rec)), **arr)
        print(json.dumps({k: v for k, v in rec.items() if not k.startswith("sd:")}, indent=None)[:2000])
        return
    ref = np.load(OUT)
    cont = json.loads(str(ref["rec"]))
    threads = min(16, len(os.sched_getaffinity(0)))
    rec, arr, ctx = run_cpu(threads=threads)
    report = {"box_cpu_capability": rec["cpu_capability"], "container_cpu_capability": cont["cpu_capability"],
              "box_threads": rec["torch_threads"], "container_threads": cont["torch_threads"],
              "box_x_after_21_equals_golden_snapshot1": rec["x_after_21_equals_golden_snapshot1"],
              "box_dev_vs_golden_fp64": rec["x_after_21_dev_vs_golden_fp64"],
              "container_dev_vs_golden_fp64": cont["x_after_21_dev_vs_golden_fp64"]}
    order = ["sd"] + sorted(k for k in cont if k.startswith("sd:")) + ["b_t", "a_t", "ab_t", "coef", "sa", "sb", "params",
                                                                       "x_T"]
    for k in range(NSTEPS):
        order += [f"{n}_{k}" for n in ("t", "z", "sc_w", "sc_b", "eps", "x")]
    diffs = [k for k in order if cont.get(k) != rec.get(k)]
    report["differing"] = diffs[:40]
    report["first_differing"] = diffs[0] if diffs else None
    per_step = []
    hip_eps, hip_x, hip_rec = (None, None, {})
    if torch.cuda.is_available():
        hip_eps, hip_x, hip_rec = run_hip(ctx)
    report.update(hip_rec)
    for k in range(NSTEPS):
        row = {"step": k, "eps_box_vs_container": _dev(arr[f"eps_{k}"], ref[f"eps_{k}"]),
               "x_box_vs_container": _dev(arr[f"x_{k}"], ref[f"x_{k}"]),
               "eps_box_ndiff": int((arr[f"eps_{k}"] != ref[f"eps_{k}"]).sum()),
               "x_box_ndiff": int((arr[f"x_{k}"] != ref[f"x_{k}"]).sum())}
        if hip_eps is not None:
            row.update({"eps_hip_vs_box": _dev(hip_eps[k], arr[f"eps_{k}"]),
                        "eps_hip_vs_container": _dev(hip_eps[k], ref[f"eps_{k}"]),
                        "x_hip_vs_box": _dev(hip_x[k], arr[f"x_{k}"]),
                        "x_hip_vs_container": _dev(hip_x[k], ref[f"x_{k}"]),
                        "x_hip_ndiff_vs_box": int((hip_x[k] != arr[f"x_{k}"]).sum())})
        per_step.append(row)
    report["per_step"] = per_step
    # the quantity that dominates the snapshot deviation: for the worst pixel of the box x after 21 steps
    print(json.dumps(report, indent=1))


if __name__ == "__main__":
    main()
