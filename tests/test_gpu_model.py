"""Whole-model parity of the HIP ContextUnet against the CPU oracle / reference golden vectors.

The tests marked MATH run with the three fp32-class 3x3-conv arithmetics: "fp32" (fp32 MFMA), "x6" (split-bf16
MFMA, 6 cross terms) and "h3" (scaled split-fp16 MFMA, 3 cross terms) — same tolerances, so x6 and h3 are held to
the fp32 bar; the fp64-anchored gradient test runs the shipped arithmetics fp32 and h3 (round 6: x6 is not shipped).

Tolerances (fp32 everywhere; only summation order differs):
  forward eps            max|d| <= 1e-4 * max|ref|
  parameter gradients    per tensor  max|d| <= 2e-3 * max|ref| + 1e-4 * max over all grads of max|ref|
  BN running stats       max|d| <= 1e-5 * max|ref| + 1e-6
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import ref_cpu as R

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


MATH = pytest.mark.parametrize("math", ["fp32", "x6", "h3"])


def _model(nf, ncf=6, sd=None, seed=0, math="fp32"):
    from cdm_amd import ContextUnet
    torch.manual_seed(seed)
    m = ContextUnet(1, nf, ncf, 64, conv_math=math)
    if sd is not None:
        m.load_state_dict({k: torch.as_tensor(v) for k, v in sd.items()})
    return m.cuda()


def _fx(name):
    return np.load(os.path.join(GOLD, name))


def _sd(fx, prefix="sd."):
    return {k[len(prefix):]: torch.from_numpy(fx[k].copy()) for k in fx.files if k.startswith(prefix)}


def _rel(got, ref):
    got = got.detach().float().cpu(); ref = ref.detach().float().cpu()
    return (got - ref).abs().max().item() / max(ref.abs().max().item(), 1e-30)


@MATH
@pytest.mark.parametrize("nf", [8, 16])
def test_eval_forward_matches_reference(nf, math):
    fx = _fx(f"model_nf{nf}.npz")
    m = _model(nf, sd=_sd(fx), math=math).eval()
    x, t, c = (torch.from_numpy(fx[k]).cuda() for k in ("x", "t", "c"))
    with torch.no_grad():
        torch.manual_seed(11)                 # the reference drew its shortcut from this seed
        eps = m(x, t, c)
        assert _rel(eps, torch.from_numpy(fx["eval_eps"])) < 1e-4
        torch.manual_seed(12)
        t1 = torch.tensor([0.37])[:, None, None, None].cuda()
        eps = m(x, t1, None)
        assert _rel(eps, torch.from_numpy(fx["eval_uncond_eps"])) < 1e-4


@MATH
def test_train_step_grads_match_reference(math):
    fx = _fx("model_nf8.npz")
    nf, T = 8, int(fx["train_T"])
    m = _model(nf, sd=_sd(fx), math=math).train()
    c = torch.from_numpy(fx["c"]).cuda()
    xp = torch.from_numpy(fx["train0_xpert"]).cuda()
    noise = torch.from_numpy(fx["train0_noise"]).cuda()
    tt = torch.from_numpy(fx["train0_t"]).cuda()
    torch.manual_seed(100)
    torch.randn(fx["x"].shape); torch.randint(1, T + 1, (fx["x"].shape[0],))  # replay the RNG order of the loop
    pred = m(xp, tt / T, c)
    loss = F.mse_loss(pred, noise)
    loss.backward()
    assert _rel(pred, torch.from_numpy(fx["train0_eps"])) < 1e-4
    assert abs(loss.item() - float(fx["train0_loss"])) <= 1e-5 * float(fx["train0_loss"])
    gmax = max(np.abs(fx["train0_grad." + k]).max() for k, _ in m.named_parameters())
    worst = []
    for k, p in m.named_parameters():
        ref = torch.from_numpy(fx["train0_grad." + k])
        err = (p.grad.cpu() - ref).abs().max().item()
        bound = 2e-3 * ref.abs().max().item() + 1e-4 * gmax
        worst.append((err / bound, k, err, ref.abs().max().item()))
        assert err <= bound, f"{k}: err {err:.3e} bound {bound:.3e}"
    print("worst grad ratios", sorted(worst)[-5:])


def test_running_stats_update():
    fx = _fx("model_nf8.npz")
    sd = _sd(fx)
    m = _model(8, sd=sd).train()
    x, t, c = (torch.from_numpy(fx[k]).cuda() for k in ("x", "t", "c"))
    with torch.no_grad():
        torch.manual_seed(5)
        m(x, t, c)
    osd = R.clone_sd(sd)
    torch.manual_seed(5)
    R.unet_forward(osd, x.cpu(), t.cpu(), c.cpu(), n_feat=8, n_cfeat=6, height=64, train=True,
                   shortcut=lambda: R.draw_shortcut(1, 8))
    for k, v in m.state_dict().items():
        if "running" in k or "num_batches" in k:
            ref = osd[k].float()
            err = (v.cpu().float() - ref).abs().max().item()
            assert err <= 1e-5 * ref.abs().max().item() + 1e-6, k


@MATH
@pytest.mark.parametrize("nf,B", [(64, 3), (128, 2)])
def test_forward_random_weights_vs_oracle(nf, B, math):
    m = _model(nf, seed=3, math=math)
    g = torch.Generator().manual_seed(9)
    x = torch.rand(B, 1, 64, 64, generator=g); t = torch.rand(B, generator=g); c = torch.rand(B, 6, generator=g)
    sd = R.clone_sd(m.state_dict())
    for train in (False, True):
        m.train(train)
        with torch.no_grad():
            torch.manual_seed(21)
            eps = m(x.cuda(), t.cuda(), c.cuda())
        torch.manual_seed(21)
        ref = R.unet_forward(R.clone_sd(sd), x, t, c, n_feat=nf, n_cfeat=6, height=64, train=train,
                             shortcut=lambda: R.draw_shortcut(1, nf))
        assert _rel(eps, ref) < 2e-4, (train, _rel(eps, ref))


def _oracle_grads(sd, x, c, noise, tt, T, ab, nf, dtype, seed, kinks=None):
    """the oracle train step (perturb + forward + mse + backward) -> (pred, grads); kinks: a _kinks.Kinks context
    around it (capture the branch, or impose one)"""
    import contextlib
    s = {k: (v.to(dtype) if v.is_floating_point() else v.clone()) for k, v in sd.items()}
    tr = R.OracleTrainer(s, n_feat=nf, n_cfeat=6, height=64)
    torch.manual_seed(seed)
    w, b = R.draw_shortcut(1, nf)
    with (kinks if kinks is not None else contextlib.nullcontext()):
        _, pred, grads = tr.step(x.to(dtype), c.to(dtype), noise.to(dtype), tt, T, ab.to(dtype),
                                 (w.to(dtype), b.to(dtype)))
    return pred, grads


_ORACLE_CACHE = {}


@pytest.mark.parametrize("math", ["fp32", "h3"])
@pytest.mark.parametrize("nf", [64, 128])
def test_train_grads_random_weights_vs_fp64(nf, math):
    """HIP grads vs an fp64 oracle, at the accuracy the reference's own fp32 CPU path has (n_feat 64 and the
    C2 width 128, where all 12 fused BN-backward layers run under h3).

    With ReLU + MaxPool, last-bit differences flip kink decisions at |z| ~ 1e-6 (either arithmetic may take either
    side; each flip reroutes a gradient upstream — relative L2 1e-3 .. 1e-2 vs a run that did not flip).  Round 5
    compares each arithmetic on its own branch (tests/_kinks.py): HIP vs fp64 autograd with HIP's decisions imposed,
    the reference's fp32 run vs fp64 with its own decisions imposed — the larger of its runs on this host's threads and
    on one thread (other CPU reduction orders).  Criterion per tensor: HIP <= 3x the reference + 2e-6; median over
    tensors <= 3x the reference's median.  Conv biases feeding a BatchNorm have an analytic gradient of 0 (rounding
    noise only): |g| <= 1e-4 * max grad.  The decisions each flips relative to plain fp64 are recorded.
    Round 6: x6 (a non-shipped arithmetic: no bench leg or config runs it) is out of this test's matrix instead of being
    held to the 5x per tensor its 20-layer backward needed at n_feat 128 (its single-conv error is up to 2x torch's own,
    DESIGN §3.1); its forward stays in the forward tests at the same bars as h3 and fp32.
    """
    import _parity
    from _kinks import Kinks, hip_kinks
    B, T = 2, 1500
    seed = {64: 4, 128: 14}[nf]
    m = _model(nf, seed=seed, math=math).train()
    sd = R.clone_sd(_model(nf, seed=seed, math=math).state_dict())
    g = torch.Generator().manual_seed(10)
    x = torch.rand(B, 1, 64, 64, generator=g); noise = torch.randn(B, 1, 64, 64, generator=g)
    c = torch.rand(B, 6, generator=g); tt = torch.randint(1, T + 1, (B,), generator=g)
    _, _, ab = R.make_schedule(T)
    xp = R.perturb_input(x, tt, noise, ab)
    torch.manual_seed(33)
    pred = m(xp.cuda(), (tt / T).cuda(), c.cuda())
    F.mse_loss(pred, noise.cuda()).backward()
    if nf not in _ORACLE_CACHE:
        refs = []
        nthreads = torch.get_num_threads()
        try:
            for th in (nthreads, 1):
                torch.set_num_threads(th)
                cap = Kinks()
                _, g32 = _oracle_grads(sd, x, c, noise, tt, T, ab, nf, torch.float32, 33, cap)
                _, g64r = _oracle_grads(sd, x, c, noise, tt, T, ab, nf, torch.float64, 33, Kinks(cap.relu, cap.pool))
                refs.append((g32, g64r))
        finally:
            torch.set_num_threads(nthreads)
        cap64 = Kinks()
        _oracle_grads(sd, x, c, noise, tt, T, ab, nf, torch.float64, 33, cap64)
        _ORACLE_CACHE[nf] = (refs, cap64)
    refs, cap64 = _ORACLE_CACHE[nf]
    torch.manual_seed(33)
    sc = R.draw_shortcut(1, nf)
    m.load_state_dict(sd)
    hk_relu, hk_pool = hip_kinks(m, xp, tt / T, c, sc, frozen=False)
    p64, g64 = _oracle_grads(sd, x, c, noise, tt, T, ab, nf, torch.float64, 33, Kinks(hk_relu, hk_pool))
    assert _rel(pred.double(), p64) < 2e-4
    flips = sum(int((a[0] != b[0]).sum()) for a, b in zip(hk_relu, cap64.relu)) + \
        sum(int((a != b).sum()) for a, b in zip(hk_pool, cap64.pool))
    gmax = max(v.abs().max().item() for v in g64.values())
    bad, errs, errs32 = [], [], []
    for k, p in m.named_parameters():
        ref = g64[k]
        got = p.grad.cpu().double()
        if ".conv1.0.bias" in k or ".conv2.0.bias" in k:
            ok = got.abs().max().item() <= 1e-4 * gmax
        else:
            e_hip = ((got - ref).norm() / ref.norm()).item()
            e_cpu = max(((g32[k].double() - g64r[k]).norm() / g64r[k].norm()).item() for g32, g64r in refs)
            ok = e_hip <= 3 * e_cpu + 2e-6
            errs.append(e_hip); errs32.append(e_cpu)
            print(f"{k:40s} l2rel hip {e_hip:.2e} cpu32 {e_cpu:.2e}")
        if not ok:
            bad.append(k)
    print(f"nf={nf} [{math}]: HIP flips {flips} decisions vs plain fp64; on each run's own branch: median rel L2 hip "
          f"{np.median(errs):.2e} (reference fp32 {np.median(errs32):.2e}), max hip {max(errs):.2e} (reference fp32 "
          f"{max(errs32):.2e})")
    _parity.record("train_grads_branch", nf=nf, conv_math=math, flips_hip=flips, hip_median=float(np.median(errs)),
                   ref32_median=float(np.median(errs32)), hip_max=max(errs), ref32_max=max(errs32))
    assert not bad, bad
    assert float(np.median(errs)) <= 3 * float(np.median(errs32))


def test_fused_bn_bwd_matches_unfused_nf128():
    """h3 at n_feat=128 (every 128/256-channel BN layer at 32^2 / 64^2 fuses its BN backward into the conv
    staging) vs the same engine with the fusion switched off (separate apply kernel, as $CDM_FUSE_BN_BWD=0).  The operands are bit-identical
    (test_bn_bwd_fused_into_conv_staging_bit_exact); only the h3 scale of dy differs (a bound on max|dy| instead
    of the measured max), i.e. the split rounding: relative L2 per gradient <= 1e-2 (the ReLU/MaxPool kink
    flips of test_train_grads_random_weights_nf64), median <= 1e-4."""
    nf, B, T = 128, 2, 1500
    g = torch.Generator().manual_seed(12)
    x = torch.rand(B, 1, 64, 64, generator=g); noise = torch.randn(B, 1, 64, 64, generator=g)
    c = torch.rand(B, 6, generator=g); tt = torch.randint(1, T + 1, (B,), generator=g)
    _, _, ab = R.make_schedule(T)
    xp = R.perturb_input(x, tt, noise, ab)
    import cdm_amd.model as M
    eng = M.get_engine(nf, 6, 64, torch.device("cuda", torch.cuda.current_device()), "h3")
    grads = []
    try:
        for fuse in (True, False):
            eng.fuse_bn_bwd = fuse
            M._WS.clear()                                  # workspaces carry the fused wiring
            m = _model(nf, seed=6, math="h3").train()
            torch.manual_seed(34)
            pred = m(xp.cuda(), (tt / T).cuda(), c.cuda())
            F.mse_loss(pred, noise.cuda()).backward()
            grads.append({k: p.grad.detach().double().cpu() for k, p in m.named_parameters()})
            if fuse:
                # the 128/256-ch BN layers with C_in > 1 whose apply is a plain BN-ReLU (dense, plain, resid)
                assert len(eng.workspace(B, True).fused) == 14
    finally:
        eng.fuse_bn_bwd = True
        M._WS.clear()
    errs = []
    for k, ref in grads[1].items():
        if ".conv1.0.bias" in k or ".conv2.0.bias" in k or ref.norm() == 0:
            continue
        errs.append(((grads[0][k] - ref).norm() / ref.norm()).item())
    print("fused vs unfused rel L2: max %.2e median %.2e" % (max(errs), float(np.median(errs))))
    assert max(errs) <= 1e-2 and float(np.median(errs)) <= 1e-4


def test_eval_forward_under_grad_mode():
    """model.eval(); model(x, t, c) outside torch.no_grad() works as in the reference and is differentiable: the
    train-structured forward with BatchNorm frozen on the running statistics (its gradients:
    tests/test_gpu_input_grads.py::test_eval_mode_grads_vs_autograd).  Same output as the folded no_grad eval path up
    to fp32 rounding, running statistics untouched, and a backward that runs."""
    fx = _fx("model_nf8.npz")
    m = _model(8, sd=_sd(fx)).eval()
    x, t, c = (torch.from_numpy(fx[k]).cuda() for k in ("x", "t", "c"))
    run0 = {k: v.clone() for k, v in m.state_dict().items() if "running" in k or "num_batches" in k}
    torch.manual_seed(11)
    out = m(x, t, c)
    assert out.requires_grad
    assert _rel(out, torch.from_numpy(fx["eval_eps"])) < 1e-4
    torch.manual_seed(11)
    with torch.no_grad():
        ref = m(x, t, c)
    assert _rel(out.detach(), ref) < 1e-5
    out.sum().backward()
    assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in m.parameters())
    for k, v in m.state_dict().items():
        if k in run0:
            assert torch.equal(v, run0[k]), k


@pytest.mark.parametrize("B", [2, 5])
def test_fused_bn_fwd_bit_exact_nf128(B):
    """h3 train at n_feat=128: the 13 dense BatchNorm + ReLU applies (incl. the C_in = 1 init conv's, whose max / min
    come from its statistics pass) fused into the next conv's staging (forward and
    weight gradient; z never written; its h3 scale from the producer's per-channel max / min) == the separate apply
    kernel ($CDM_FUSE_BN_FWD=0), bit for bit: output, every gradient, BatchNorm running statistics."""
    nf, T = 128, 1500
    g = torch.Generator().manual_seed(15)
    x = torch.rand(B, 1, 64, 64, generator=g); noise = torch.randn(B, 1, 64, 64, generator=g)
    c = torch.rand(B, 6, generator=g); tt = torch.randint(1, T + 1, (B,), generator=g)
    _, _, ab = R.make_schedule(T)
    xp = R.perturb_input(x, tt, noise, ab)
    import cdm_amd.model as M
    eng = M.get_engine(nf, 6, 64, torch.device("cuda", torch.cuda.current_device()), "h3")
    res = []
    sums0 = eng.fuse_bn_sums
    eng.fuse_bn_sums = False      # (the producer sums ride on the fused X staging: same sums, other summation order)
    try:
        for fuse in (True, False):
            eng.fuse_bn_fwd = fuse
            M._WS.clear()
            m = _model(nf, seed=16, math="h3").train()
            torch.manual_seed(35)
            pred = m(xp.cuda(), (tt / T).cuda(), c.cuda())
            F.mse_loss(pred, noise.cuda()).backward()
            ws = eng.workspace(B, True)
            assert len(ws.fused_fwd) == (13 if fuse else 0)
            res.append((pred.detach().cpu(), {k: p.grad.detach().cpu() for k, p in m.named_parameters()},
                        {k: v.detach().cpu() for k, v in m.state_dict().items() if "running" in k}))
    finally:
        eng.fuse_bn_fwd = True
        eng.fuse_bn_sums = sums0
        M._WS.clear()
    assert torch.equal(res[0][0], res[1][0])
    for k in res[1][1]:
        assert torch.equal(res[0][1][k], res[1][1][k]), k
    for k in res[1][2]:
        assert torch.equal(res[0][2][k], res[1][2][k]), k


@pytest.mark.parametrize("math", ["h3", "bf16"])
def test_bn_sums_in_consumer_wgrad_nf128(math):
    """The BatchNorm-backward channel sums of each fused dense producer computed in its consumer's weight-gradient X
    staging (PreBnReluSums, one partial per block; the default since round 4) vs the separate
    cdm_norm_bwd_reduce pass, n_feat
    128, B=3: the forward (eps, running statistics) is untouched (bit-identical); the gradients differ only by the sums'
    fp32 summation order, which moves the BN-backward coefficients by rounding: relative L2 per gradient <= 1e-2 (the
    kink flips of test_train_grads_random_weights_vs_fp64), median <= 1e-4 under h3; under bf16 a last-bit change of
    a coefficient flips the bf16 rounding of dy elements, so max <= 5e-2, median <= 5e-3 (the bf16 operand noise of
    the reference itself is ~0.3 relative L2 median on such gradients, test_c4_bf16_train_grads_vs_fp64; measured
    1.25e-2 / 2.0e-3)."""
    nf, B, T = 128, 3, 1500
    g = torch.Generator().manual_seed(17)
    x = torch.rand(B, 1, 64, 64, generator=g); noise = torch.randn(B, 1, 64, 64, generator=g)
    c = torch.rand(B, 6, generator=g); tt = torch.randint(1, T + 1, (B,), generator=g)
    _, _, ab = R.make_schedule(T)
    xp = R.perturb_input(x, tt, noise, ab)
    import cdm_amd.model as M
    eng = M.get_engine(nf, 6, 64, torch.device("cuda", torch.cuda.current_device()), math)
    res = []
    sums0, act0 = eng.fuse_bn_sums, eng.act16
    eng.act16 = False        # bf16 activations need the fused sums (the separate pass reads fp32 y / g): fp32 both ways
    try:
        for on in (True, False):
            eng.fuse_bn_sums = on
            M._WS.clear()
            m = _model(nf, seed=18, math=math).train()
            torch.manual_seed(36)
            pred = m(xp.cuda(), (tt / T).cuda(), c.cuda())
            F.mse_loss(pred, noise.cuda()).backward()
            ws = eng.workspace(B, True)
            assert len(ws.sums_from) == (13 if on else 0), sorted(ws.sums_from)
            res.append((pred.detach().cpu(), {k: p.grad.detach().double().cpu() for k, p in m.named_parameters()},
                        {k: v.detach().cpu() for k, v in m.state_dict().items() if "running" in k}))
    finally:
        eng.fuse_bn_sums, eng.act16 = sums0, act0
        M._WS.clear()
    assert torch.equal(res[0][0], res[1][0])
    for k in res[1][2]:
        assert torch.equal(res[0][2][k], res[1][2][k]), k
    errs = []
    for k, ref in res[1][1].items():
        if ".conv1.0.bias" in k or ".conv2.0.bias" in k or ref.norm() == 0:
            continue
        errs.append(((res[0][1][k] - ref).norm() / ref.norm()).item())
    print(f"[{math}] sums in wgrad vs separate pass: rel L2 max {max(errs):.2e} median {float(np.median(errs)):.2e}")
    if math == "h3":
        assert max(errs) <= 1e-2 and float(np.median(errs)) <= 1e-4
    else:
        assert max(errs) <= 5e-2 and float(np.median(errs)) <= 5e-3


def test_eval_pack_not_shared_across_models():
    """Models of one shape share an engine and its packed eval weights; a model created after another was freed can
    get the freed model's tensor addresses with the same version counters.  Its eval forward must still run on its own
    weights (the pack key carries the model's identity): ten models of different seeds, each freed before the next
    is built, each eval forward vs the oracle on that model's weights."""
    import gc
    g = torch.Generator().manual_seed(3)
    x = torch.rand(2, 1, 64, 64, generator=g); t = torch.rand(2, generator=g); c = torch.rand(2, 6, generator=g)
    for seed in range(10):
        m = _model(16, seed=100 + seed, math="h3").eval()
        sd = R.clone_sd(m.state_dict())
        with torch.no_grad():
            torch.manual_seed(5)
            eps = m(x.cuda(), t.cuda(), c.cuda())
        torch.manual_seed(5)
        ref = R.unet_forward(sd, x, t, c, n_feat=16, n_cfeat=6, height=64, train=False,
                             shortcut=lambda: R.draw_shortcut(1, 16))
        assert _rel(eps, ref) < 2e-4, seed
        del m, eps
        gc.collect()


@pytest.mark.parametrize("math", ["h3", "bf16"])
def test_eval_fused_epilogue_matches_apply_kernel(math):
    """The eval forward's residual / FiLM / MaxPool applies in the conv epilogue (cdm_conv3x3_fwd_x16_fused,
    engine.fuses_eval) vs the conv + cdm_norm_apply_fwd pair they replace, n_feat = 128 (the fused shapes: 64^2 residual
    and pool, 32^2 FiLM and pool), per-sample t / c and a broadcast t: the same values (bit-identical or within
    1e-6 of max|eps|; recorded), and a CFG sampling run (two shortcut sets, the batched 2n forward) likewise."""
    import cdm_amd
    from cdm_amd.diffusion import GraphSampler, Schedule
    m = _model(128, math=math).eval()
    eng, _ = m._engine_and_params()
    assert eng.fuse_eval
    g = torch.Generator().manual_seed(12)
    x = torch.randn(3, 1, 64, 64, generator=g).cuda()
    c = torch.rand(3, 6, generator=g).cuda()
    res = {}
    for tb in (torch.rand(3, generator=g).cuda(), torch.rand(1, generator=g).cuda()):
        outs = []
        for fuse in (True, False):
            eng.fuse_eval = fuse
            torch.manual_seed(7)
            with torch.no_grad():
                outs.append(m(x, tb, c).cpu())
        d = (outs[0] - outs[1]).abs().max().item() / outs[1].abs().max().item()
        res[f"t_rows_{tb.numel()}"] = d
        assert d <= 1e-6, d
    params = torch.rand(2, 6, generator=torch.Generator().manual_seed(3))
    sched = Schedule(12, "cuda")
    xs = []
    for fuse in (True, False):
        eng.fuse_eval = fuse
        smp = GraphSampler(m, sched, 2, 3.0, params, z_source="device", seed=5, use_graph=False)
        torch.manual_seed(4)
        smp.prepare_rng(host_z=False)
        xT = torch.randn(2, 1, 64, 64, generator=torch.Generator().manual_seed(2))
        xs.append(smp.run(xT)[0].cpu())
    eng.fuse_eval = True
    d = (xs[0] - xs[1]).abs().max().item() / xs[1].abs().max().item()
    res["cfg_sample"] = d
    print(math, "fused vs apply kernel, max rel diff:", res)
    assert d <= 1e-5, d


@pytest.mark.parametrize("H", [20, 36, 48])
def test_map_heights_not_multiple_of_16(H):
    """ContextUnet(height=H) for any H % 4 == 0 (the reference's only requirement: ContextUnet.py:17,27 — two MaxPool2d(2),
    AvgPool2d(H/4), ConvTranspose2d(k = H/4)); widths outside the LDS-halo / band kernels' set run the generic kernels
    (split GEMM convs, fp32 weight-gradient GEMMs for widths % 8 != 0).  n_feat 16, B 2, h3: forward train / eval vs
    the fp32 oracle (2e-4) and every parameter gradient vs fp64 at the bar of test_train_grads_random_weights_vs_fp64
    (it was an absolute 1e-2 / 5e-3): each run on its own ReLU / MaxPool branch (tests/_kinks.py), per tensor
    HIP <= 3x the reference fp32 run's relative L2 + 2e-6, median over tensors <= 3x the reference's median."""
    from cdm_amd import ContextUnet
    from _kinks import Kinks, hip_kinks
    nf, B, T = 16, 2, 1500
    torch.manual_seed(23)
    m = ContextUnet(1, nf, 6, H).cuda()
    sd = R.clone_sd(m.state_dict())
    g = torch.Generator().manual_seed(31)
    x = torch.rand(B, 1, H, H, generator=g); noise = torch.randn(B, 1, H, H, generator=g)
    c = torch.rand(B, 6, generator=g); tt = torch.randint(1, T + 1, (B,), generator=g)
    for train in (False, True):
        m.train(train)
        with torch.no_grad():
            torch.manual_seed(21)
            eps = m(x.cuda(), (tt / T).cuda(), c.cuda())
        torch.manual_seed(21)
        ref = R.unet_forward(R.clone_sd(sd), x, tt / T, c, n_feat=nf, n_cfeat=6, height=H, train=train,
                             shortcut=lambda: R.draw_shortcut(1, nf))
        assert _rel(eps, ref) < 2e-4, (H, train, _rel(eps, ref))
    m.load_state_dict(sd)
    m.train()
    _, _, ab = R.make_schedule(T)
    xp = R.perturb_input(x, tt, noise, ab)
    torch.manual_seed(33)
    pred = m(xp.cuda(), (tt / T).cuda(), c.cuda())
    F.mse_loss(pred, noise.cuda()).backward()
    torch.manual_seed(33)
    sc = R.draw_shortcut(1, nf)                      # the draw the module made
    got = {k: p.grad.cpu().double() for k, p in m.named_parameters()}
    m.load_state_dict(sd)
    hk_relu, hk_pool = hip_kinks(m, xp, tt / T, c, sc, frozen=False)

    def oracle(dtype, kinks):
        s = {k: (v.to(dtype) if v.is_floating_point() else v.clone()) for k, v in sd.items()}
        tr = R.OracleTrainer(s, n_feat=nf, n_cfeat=6, height=H)
        with kinks:
            return tr.step(x.to(dtype), c.to(dtype), noise.to(dtype), tt, T, ab.to(dtype),
                           (sc[0].to(dtype), sc[1].to(dtype)))
    _, p64, g64 = oracle(torch.float64, Kinks(hk_relu, hk_pool))
    cap32 = Kinks()
    _, _, g32 = oracle(torch.float32, cap32)
    _, _, g64r = oracle(torch.float64, Kinks(cap32.relu, cap32.pool))
    assert _rel(pred.double(), p64) < 2e-4
    gmax = max(v.abs().max().item() for v in g64.values())
    errs, errs32, bad = {}, {}, []
    for k, v in got.items():
        if ".conv1.0.bias" in k or ".conv2.0.bias" in k:
            assert v.abs().max().item() <= 1e-4 * gmax, k
            continue
        errs[k] = ((v - g64[k]).norm() / g64[k].norm()).item()
        errs32[k] = ((g32[k].double() - g64r[k]).norm() / g64r[k].norm()).item()
        if errs[k] > 3 * errs32[k] + 2e-6:
            bad.append((k, errs[k], errs32[k]))
    med, med32 = float(np.median(list(errs.values()))), float(np.median(list(errs32.values())))
    print(f"H={H}: grads vs fp64 (own branches) max {max(errs.values()):.2e} median {med:.2e}; reference fp32 max "
          f"{max(errs32.values()):.2e} median {med32:.2e}")
    assert not bad, bad
    assert med <= 3 * med32
