"""End-to-end parity of the benchmarked C4 configuration (BASELINE configs[3]: bf16 mixed-precision training): the Trainer
step bench.py times for C4, at its own shape — n_feat = 128, 6 params, 64x64, B = 256, T = 1500, conv_math = "bf16",
hipGraph replay; the first two bench steps (seeded init torch.manual_seed(0), x0 / c from the CUDA generator 1234,
Trainer seed 0, lr 1e-5, Philox noise / t / shortcut read back from the Trainer's device buffers).

The reference for mixed precision is the reference run under torch.autocast-like rounding: the CPU oracle with every 3x3
conv (C_in > 1) and both ConvTranspose2d(2, 2) taking bf16-rounded operands, fp32 accumulate, and those 3x3 convs'
outputs and their gradients stored in bf16 (test_gpu_configs._bf16_operands(outputs=True); the HIP step stores the fused
chain's y and g in bf16) — and the truth is the oracle in fp64
(tests/_oracle_gpu.py, on the GPU).  Bar, per step: HIP's deviation from fp64 within 1.5x the emulated reference's
  eps            max|d| / max|eps|
  loss           |d|                                       (+ 1e-7 |loss|)
  gradients      relative L2 per tensor: max and median over tensors (BN-fed conv biases: |g| <= 1e-3 max|g|)
  parameters     after Adam, |dp| / lr: RMS and 99th percentile (step 1; step 2's oracles would start a fresh Adam)
and the fused Adam equal to the restatement of torch.optim.Adam on >= 99.999 % of the parameters, moments bit-exact.
Step 1 is the eager first step, step 2 the captured graph's replay (from HIP's state after step 1).
Reference: code/train_diffusion_condition.py:216-230, code/diffusion_utilities.py:26-37.
"""
import numpy as np
import pytest
import torch

import _oracle_gpu
import _parity
from oracle import ref_cpu as R

pytestmark = pytest.mark.gpu
NF, NCF, H, B, T, LR = 128, 6, 64, 256, 1500, 1e-5


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    old = torch.get_num_threads()
    torch.set_num_threads(min(16, max(1, len(__import__("os").sched_getaffinity(0)))))
    yield
    torch.set_num_threads(old)


def _bn_fed_bias(k):
    return ".conv1.0.bias" in k or ".conv2.0.bias" in k


_HIP = {}


def _flat_views(tr, flat):
    out = {}
    for n, view in tr.views.items():
        lo = (view.data_ptr() - tr.flat.data_ptr()) // 4
        out[n] = flat[lo:lo + view.numel()].view_as(view)
    return out


def _hip_steps():
    if _HIP:
        return _HIP
    from cdm_amd import ContextUnet, Trainer
    torch.manual_seed(0)
    m = ContextUnet(1, NF, NCF, H, shortcut_source="device", conv_math="bf16").cuda()
    sd0 = R.clone_sd(m.state_dict())
    tr = Trainer(m, LR, T, B, seed=0, use_graph=True)
    g = torch.Generator(device="cuda").manual_seed(1234)
    x0 = torch.rand(B, 1, H, H, device="cuda", generator=g)
    c = torch.rand(B, NCF, device="cuda", generator=g)
    steps = []
    for k in range(2):
        pre = (tr.flat.cpu(), tr.m.cpu(), tr.v.cpu())
        loss = float(tr.step(x0, c).item())
        torch.cuda.synchronize()
        sb = tr.cur
        steps.append(dict(
            step=k + 1, replay=tr.graph is not None and k == 1, loss=loss,
            noise=sb.noise.view(B, 1, H, H).cpu().clone(), t=sb.t_int.cpu().long().clone(), sc=tr.sc.cpu().clone(),
            eps=sb.ws.eps.view(B, 1, H, H).cpu().clone(), gflat=tr.gflat.cpu().clone(),
            pre=pre, post=(tr.flat.cpu(), tr.m.cpu(), tr.v.cpu()),
            sd={kk: v.detach().cpu().clone() for kk, v in m.state_dict().items()}))
    assert steps[1]["replay"], "step 2 must be the captured graph's replay"
    _HIP.update(sd0=sd0, x=x0.cpu(), c=c.cpu(), steps=steps, tr=tr)
    return _HIP


def _emulated_step(sd, x, c, st):
    """The reference's fp32 step under bf16 operand rounding (CPU oracle: the reference's arithmetic)."""
    from test_gpu_configs import _bf16_operands
    s = {k: (v.float() if v.is_floating_point() else v.clone()) for k, v in sd.items()}
    otr = R.OracleTrainer(s, n_feat=NF, n_cfeat=NCF, height=H, lr=LR)
    _, _, ab = R.make_schedule(T)
    w = st["sc"][:NF].reshape(NF, 1, 1, 1).float(); b = st["sc"][NF:].float()
    with _bf16_operands(outputs=True):
        loss, pred, grads = otr.step(x, c, st["noise"], st["t"], T, ab, (w, b))
    return float(loss), pred.detach(), grads, {k: v.detach().clone() for k, v in otr.sd.items()}


def _metrics(tr, st, got_post, emu, f64):
    """HIP and emulated-reference deviations from fp64 (eps, loss, gradients, parameters after Adam)."""
    le, pe, ge, se = emu
    l64, p64, g64, s64 = f64
    mx = p64.abs().max().item()
    hip_g = {n: v.clone() for n, v in _flat_views(tr, st["gflat"]).items()}
    gmax = max(v.abs().max().item() for v in g64.values())
    eg, ee, zero = {}, {}, 0.0
    for n, r in g64.items():
        r = r.double()
        if _bn_fed_bias(n):
            zero = max(zero, hip_g[n].abs().max().item() / gmax)
            continue
        eg[n] = ((hip_g[n].double() - r).norm() / r.norm()).item()
        ee[n] = ((ge[n].double() - r).norm() / r.norm()).item()
    keep = [n for n in tr.views if not _bn_fed_bias(n)]

    def dev(post):
        d = np.concatenate([((post[n].double() - s64[n].double()) / LR).abs().numpy().ravel() for n in keep])
        return float(np.sqrt((d ** 2).mean())), float(np.percentile(d, 99))
    h_rms, h_p99 = dev(got_post)
    e_rms, e_p99 = dev(se)
    return dict(eps=(st["eps"].double() - p64).abs().max().item() / mx, eps_emu=(pe.double() - p64).abs().max().item() / mx,
                loss=abs(st["loss"] - l64), loss_emu=abs(le - l64), loss64=l64,
                grad_max=max(eg.values()), grad_max_emu=max(ee.values()),
                grad_median=float(np.median(list(eg.values()))), grad_median_emu=float(np.median(list(ee.values()))),
                dp_rms=h_rms, dp_rms_emu=e_rms, dp_p99=h_p99, dp_p99_emu=e_p99, bn_fed_bias_max_rel=zero)


def _adam_exact(st):
    p0, m0, v0 = (a.numpy() for a in st["pre"])
    p1, m1, v1 = (a.numpy() for a in st["post"])
    rp, rm, rv = R.adam_step_restated(p0, st["gflat"].numpy(), m0, v0, LR, st["step"])
    return float((p1 == rp).mean()), bool(np.array_equal(m1, rm) and np.array_equal(v1, rv))


def _check(r, name):
    print(f"C4 {name}: eps {r['eps']:.2e} (emulated bf16 reference {r['eps_emu']:.2e}); loss {r['loss']:.2e} "
          f"({r['loss_emu']:.2e}); grads max {r['grad_max']:.2e} ({r['grad_max_emu']:.2e}) median {r['grad_median']:.2e} "
          f"({r['grad_median_emu']:.2e}); |dp|/lr rms {r['dp_rms']:.2e} ({r['dp_rms_emu']:.2e}) p99 {r['dp_p99']:.2e} "
          f"({r['dp_p99_emu']:.2e}); Adam exact {r['adam_exact_frac']:.6f}")
    assert r["eps"] <= 1.5 * r["eps_emu"]
    assert r["loss"] <= 1.5 * r["loss_emu"] + 1e-7 * abs(r["loss64"])
    assert r["grad_max"] <= 1.5 * r["grad_max_emu"] and r["grad_median"] <= 1.5 * r["grad_median_emu"]
    assert r["dp_rms"] <= 1.5 * r["dp_rms_emu"] and r["dp_p99"] <= 1.5 * r["dp_p99_emu"]   # (step 1)
    assert r["bn_fed_bias_max_rel"] <= 1e-3
    assert r["adam_exact_frac"] >= 0.99999 and r["adam_moments_exact"]


def _run_step(k):
    hip = _hip_steps()
    st = hip["steps"][k]
    tr = hip["tr"]
    sd = hip["sd0"] if k == 0 else {kk: v.clone() for kk, v in hip["steps"][0]["sd"].items()}
    emu = _emulated_step(sd, hip["x"], hip["c"], st)
    f64 = _oracle_gpu.train_step(sd, hip["x"], hip["c"], st["noise"], st["t"], st["sc"], n_feat=NF, n_cfeat=NCF,
                                 height=H, T=T, lr=LR)
    r = _metrics(tr, st, _flat_views(tr, st["post"][0]), emu, f64)
    if k == 1:
        # the oracles start a fresh Adam from HIP's step-1 parameters, HIP takes Adam's second step (moments of step
        # 1): the update itself is pinned by the restatement check below, not by a parameter comparison
        for key in ("dp_rms", "dp_rms_emu", "dp_p99", "dp_p99_emu"):
            r[key] = 0.0
    r["adam_exact_frac"], r["adam_moments_exact"] = _adam_exact(st)
    return r


def test_c4_step1_vs_emulated_reference():
    r = _run_step(0)
    _parity.record("c4_e2e_step1", B=B, n_feat=NF, conv_math="bf16", **r)
    _check(r, "step 1 (eager)")


def test_c4_step2_graph_replay_vs_emulated_reference():
    r = _run_step(1)
    _parity.record("c4_e2e_step2_replay", B=B, n_feat=NF, conv_math="bf16", **r)
    _check(r, "step 2 (graph replay)")
