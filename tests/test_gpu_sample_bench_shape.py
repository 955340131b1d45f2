"""Parity of the benchmarked sampling batch: the bench's own eval path at its own size.

bench.py's sampling legs run GraphSampler (diffusion.py) at n = 256 (w = 0: one 256-image forward per step) and, for CFG,
one batched 2n = 512-image forward per step whose two halves carry the two shortcut draws of the reference's cond and
uncond calls (code/train_diffusion_condition.py:312-329).  At that size the eval convs run the fused residual / FiLM /
MaxPool epilogue (EpiStoreW<..., FUSE = true>) on multi-tile LDS-halo blocks (several 256-pixel tiles per block, the
next tile's halo prefetched into the buffer the fused epilogue's scratch lives in) — a combination the n = 2 trajectory
goldens never reach.  Checked here, for h3 (C2) and bf16 (C4), n_feat = 128, T = 1500:

  1. one denoise step's forward (step i = T, the sampler's prologue / shortcut table / t broadcast), eps of both halves
     against the oracle (oracle/ref_cpu.py, the restatement of ContextUnet.py:42-60) evaluated in fp64 on the GPU as
     the checker (tests/_oracle_gpu.py's approach), next to the reference's fp32 CPU run of the same forward on the same
     inputs (C4: the reference under C4's bf16 operand rounding, tests/_bf16emu.py);
  2. the same forward with the apply-kernel path (engine.fuse_eval off): the fused epilogue equals it (<= 1e-6 max|eps|);
  3. a 20-step segment (i = 1500 .. 1481) through the captured 10-step graphs the bench replays, with host-replayed z
     and shortcut draws, against the oracle's fp64 segment on the GPU; the reference's fp32 segment on the CPU runs on
     a 16-image subset (eval mode: images are independent, so the subset is the reference's per-image error).

Bars: h3 — max|d| / max|ref64| within 3x the reference fp32's, relative L2 within 3x; bf16 — relative L2 within 1.5x
the bf16-emulated reference's (the C4 bar of tests/test_gpu_configs.py).  Whole-batch relative L2 vs the subset's
reference relative L2 (an RMS statistic, independent of the image count).  Measured values -> $CDM_PARITY_OUT.
The denoise update itself is bit-exact vs the reference's fp32 ops (test_gpu_sampler.py::test_perturb_and_denoise_
bit_exact); the oracle segments below apply it with the Schedule's coefficient tables, so only the network differs."""
import os

import numpy as np
import pytest
import torch

from oracle import ref_cpu as R
import _parity

pytestmark = pytest.mark.gpu
NF, NCF, H, T, N = 128, 6, 64, 1500, 256
SEG, SUB = 20, 16              # segment length (two captured 10-step graphs); reference fp32 subset (images)


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    old = torch.get_num_threads()
    torch.set_num_threads(min(16, max(1, len(os.sched_getaffinity(0)))))
    yield
    torch.set_num_threads(old)


def _model(math):
    """Seeded default init (bench.py's torch.manual_seed(0)) with non-trivial BatchNorm running statistics (the eval
    forward folds them into the packed weights)."""
    from cdm_amd import ContextUnet
    torch.manual_seed(0)
    m = ContextUnet(1, NF, NCF, H, conv_math=math)
    g = torch.Generator().manual_seed(41)
    with torch.no_grad():
        for k, v in m.state_dict().items():
            if k.endswith("running_mean"):
                v.copy_(0.05 * torch.randn(v.shape, generator=g))
            elif k.endswith("running_var"):
                v.copy_(0.6 + 0.8 * torch.rand(v.shape, generator=g))
    sd = R.clone_sd(m.state_dict())
    return m.cuda().eval(), sd


def _draws(cfg, seed):
    """x_T, params, z of each segment step (all have i > 1) and each step's shortcut sets (cond[, uncond]), drawn as
    the reference's nn.Conv2d(1, n_feat, 1) init draws them: U(-1, 1) for weight and bias (fan_in 1)."""
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(N, 1, H, H, generator=g)
    params = torch.rand(N, NCF, generator=g)
    z = torch.randn(SEG, N, 1, H, H, generator=g)
    sets = 2 if cfg else 1
    sc = []
    for _ in range(SEG):
        ws, bs = [], []
        for _ in range(sets):
            ws.append(torch.rand(NF, generator=g) * 2 - 1); bs.append(torch.rand(NF, generator=g) * 2 - 1)
        sc.append((ws, bs))
    return x, params, z, sc


def _sampler(m, w, params, sc, z, use_graph):
    """GraphSampler as bench.py builds it (n = 256, save_rate 20, K = 10 steps per graph), its shortcut table and a
    z table holding this test's draws for the first SEG steps (denoise_kernel reads z_table[T - i])."""
    from cdm_amd.diffusion import GraphSampler, Schedule
    sched = Schedule(T, "cuda")
    smp = GraphSampler(m, sched, N, w, params, save_rate=20, z_source="device", seed=4321, use_graph=use_graph)
    rows = torch.zeros(T, smp.row)
    for k, (ws, bs) in enumerate(sc):
        rows[k] = torch.cat(ws + bs)
    smp.sc_table.copy_(rows)
    smp.z_table = z.reshape(SEG, N * H * H).cuda().contiguous()
    return smp, sched


def _fwd(sd, x, t, c, sc, dtype, device, bf16emu=False):
    s = {k: (v.to(dtype) if v.is_floating_point() else v.clone()).to(device) for k, v in sd.items()}
    w, b = sc
    args = dict(n_feat=NF, n_cfeat=NCF, height=H, train=False,
                shortcut=(w.reshape(NF, 1, 1, 1).to(dtype).to(device), b.to(dtype).to(device)))
    with torch.no_grad():
        if bf16emu:
            from _bf16emu import _bf16_operands
            with _bf16_operands():
                return R.unet_forward(s, x.to(dtype).to(device), t.to(dtype).to(device), c.to(dtype).to(device), **args)
        return R.unet_forward(s, x.to(dtype).to(device), t.to(dtype).to(device), c.to(dtype).to(device), **args)


def _eps_ref(sd, x, i, params, sc_step, cfg, w, dtype, device, bf16emu=False):
    """The reference's eps at step i (:318-329): cond forward, then the uncond forward with c = 0 and its own draw."""
    t = torch.tensor([i / T])
    ws, bs = sc_step
    ec = _fwd(sd, x, t, params, (ws[0], bs[0]), dtype, device, bf16emu)
    if not cfg:
        return ec, None
    eu = _fwd(sd, x, t, torch.zeros_like(params), (ws[1], bs[1]), dtype, device, bf16emu)
    return ec, eu


def _errs(got, ref):
    got, ref = got.double().cpu(), ref.double().cpu()
    return (float((got - ref).abs().max() / ref.abs().max()), float((got - ref).norm() / ref.norm()))


def _bars(math, name, e_hip, e_ref, e_hip_all=None, **rec):
    """(max, relL2) of HIP and of the reference vs fp64 -> assert the bar, record."""
    _parity.record(name, conv_math=math, hip_max=e_hip[0], hip_rel_l2=e_hip[1], ref_max=e_ref[0],
                   ref_rel_l2=e_ref[1], hip_all_rel_l2=None if e_hip_all is None else e_hip_all[1], **rec)
    print(f"{name} [{math}] {rec}: HIP max {e_hip[0]:.3e} relL2 {e_hip[1]:.3e} | reference max {e_ref[0]:.3e} relL2 "
          f"{e_ref[1]:.3e}" + ("" if e_hip_all is None else f" | HIP whole batch relL2 {e_hip_all[1]:.3e}"))
    if math == "bf16":
        assert e_hip[1] <= 1.5 * e_ref[1], (name, e_hip, e_ref)
        if e_hip_all is not None:
            assert e_hip_all[1] <= 1.5 * e_ref[1], (name, e_hip_all, e_ref)
    else:
        assert e_hip[0] <= 3 * e_ref[0] and e_hip[1] <= 3 * e_ref[1], (name, e_hip, e_ref)
        if e_hip_all is not None:
            assert e_hip_all[1] <= 3 * e_ref[1], (name, e_hip_all, e_ref)


@pytest.mark.parametrize("w", [0.0, 3.0])
@pytest.mark.parametrize("math", ["h3", "bf16"])
def test_bench_batch_forward_vs_fp64(math, w):
    """One sampler step at n = 256 (w = 0) / the batched 512-image CFG forward (w = 3): eps of every image of both halves
    vs the fp64 oracle, the reference's fp32 (C4: bf16-emulated) forward of all 256 images beside it; and the fused
    eval epilogue == the apply-kernel path at this batch."""
    cfg = w > 0
    m, sd = _model(math)
    x, params, z, sc = _draws(cfg, seed=1000 + int(w))
    smp, _ = _sampler(m, w, params, sc, z, use_graph=False)
    eng = smp.eng
    assert eng.fuse_eval and all(eng.fuses_eval(l, smp.B) for l in eng.layers
                                 if smp.ws.dst_kind[l.name] in ("pool", "film", "resid") and l.cin > 1)
    outs = {}
    for fuse in (True, False):
        eng.fuse_eval = fuse
        try:
            smp.run(x, steps=1)
        finally:
            eng.fuse_eval = True
        torch.cuda.synchronize()
        outs[fuse] = smp.ws.eps.view(smp.B, 1, H, H).cpu().clone()
    eps = outs[True]
    d_apply = float((outs[True] - outs[False]).abs().max() / outs[False].abs().max())
    ec64, eu64 = _eps_ref(sd, x, T, params, sc[0], cfg, w, torch.float64, "cuda")
    ec32, eu32 = _eps_ref(sd, x, T, params, sc[0], cfg, w, torch.float32, "cpu", bf16emu=math == "bf16")
    halves = [("cond", eps[:N], ec64, ec32)] + ([("uncond", eps[N:], eu64, eu32)] if cfg else [])
    for half, got, r64, r32 in halves:
        _bars(math, "sample_bench_batch_forward", _errs(got, r64), _errs(r32, r64), w=w, half=half, batch=smp.B,
              fused_vs_apply=d_apply)
    assert d_apply <= 1e-6, d_apply


@pytest.mark.parametrize("w", [0.0, 3.0])
@pytest.mark.parametrize("math", ["h3", "bf16"])
def test_bench_batch_segment_vs_fp64(math, w):
    """20 steps (i = 1500 .. 1481) of the bench's sampler at n = 256 — two replays of the captured 10-step graph, the
    CFG combine in the denoise kernel — from host-replayed draws, vs the oracle's segment in fp64 on the GPU; the
    reference's fp32 (C4: bf16-emulated) segment on the first 16 images beside it."""
    cfg = w > 0
    m, sd = _model(math)
    x, params, z, sc = _draws(cfg, seed=2000 + int(w))
    smp, sched = _sampler(m, w, params, sc, z, use_graph=True)
    xh, _ = smp.run(x, steps=SEG)
    assert smp.graph is not None and smp.K == 10
    xh = xh.cpu()
    coef, sa, sb = (v.cpu() for v in (sched.coef, sched.sa, sched.sb))

    def segment(dtype, device, n, bf16emu=False):
        xs = x[:n].to(dtype).to(device)
        p = params[:n]
        for k, i in enumerate(range(T, T - SEG, -1)):
            ec, eu = _eps_ref(sd, xs, i, p, sc[k], cfg, w, dtype, device, bf16emu)
            e = ec if eu is None else eu + w * (ec - eu)
            zi = z[k, :n].to(dtype).to(device)
            xs = (xs - e * coef[i].to(dtype)) / sa[i].to(dtype) + sb[i].to(dtype) * zi   # :274-279, same op order
        return xs.cpu()
    x64 = segment(torch.float64, "cuda", N)
    x32 = segment(torch.float32, "cpu", SUB, bf16emu=math == "bf16")
    _bars(math, "sample_bench_batch_segment", _errs(xh[:SUB], x64[:SUB]), _errs(x32, x64[:SUB]),
          e_hip_all=_errs(xh, x64), w=w, steps=SEG, batch=smp.B, subset=SUB, max_abs_x=float(x64.abs().max()))
