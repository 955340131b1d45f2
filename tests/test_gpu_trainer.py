"""Parity of the benchmarked training step (row a8): cdm_amd.Trainer — fused Adam, device optimizer state,
Philox / injected draws, hipGraph replay — against the reference's own training loop and torch.optim.Adam.

Golden data: tests/golden/train_nf8.npz, three iterations of the reference loop body
(code/train_diffusion_condition.py:213-229; lr 1e-3, 1e-3, then 7.5e-4 = the per-epoch decay of :213) from the
seed-0 weights of model_nf8.npz, with each step's draws (noise, t, 1x1 shortcut) recorded so the Trainer can
replay them (inject mode).

Bars (each stated where it is asserted):
  * Adam given identical gradients: cdm_adam == oracle.adam_step_restated (torch's _single_tensor_adam with the
    roundings of its CPU kernels and a correctly rounded sqrt; pinned to torch.optim.Adam on the reference's host
    by tests/test_oracle_adam.py) on >= 99.999 % of the parameters (all but fp64-emulated fma double roundings),
    exp_avg / exp_avg_sq bit-identical; vs this host's torch CPU Adam, whose vectorised sqrt rounds
    host-dependently, the moments bit-identical and every parameter within ulp(p) + 1e-3 |update|.
  * step-0 gradients vs the fp64 oracle: rel L2 median <= 5e-3, every tensor <= 2e-2 (a kink flip).
  * parameters after 1, 2, 3 steps vs the reference: Adam turns gradient noise into +-lr-sized moves (step one is
    lr * sign(g)), so the bar is anchored like test_train_grads_random_weights_nf64: the same three steps run by
    the CPU oracle in fp64 give the reference's own fp32 deviation; the HIP deviation from fp64 must stay within
    3x of it (RMS and 99th percentile of |dp| / lr over every parameter except the conv biases that feed a
    BatchNorm, whose analytic gradient is 0 and whose updates are sign noise in both: those only <= 2 lr per step).
  * graph replay == eager, bit for bit (parameters, Adam moments, BN running stats, loss), across an eval-mode
    forward between steps (the eval weight pack must be rebuilt after the in-place Adam) and an LR change.
"""
import os

import numpy as np
import pytest
import torch

from oracle import ref_cpu as R
import _parity

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _bn_fed_bias(k):
    return ".conv1.0.bias" in k or ".conv2.0.bias" in k


def _model(nf, sd=None, seed=0, math="h3"):
    from cdm_amd import ContextUnet
    torch.manual_seed(seed)
    m = ContextUnet(1, nf, 6, 64, conv_math=math)
    if sd is not None:
        m.load_state_dict({k: torch.as_tensor(v) for k, v in sd.items()})
    return m.cuda().train()


def _golden_sd(fx, prefix):
    return {k[len(prefix):]: torch.from_numpy(fx[k].copy()) for k in fx.files if k.startswith(prefix)}


def _params(tr):
    return {n: v.detach().cpu().clone() for n, v in tr.views.items()}


def _fp64_oracle_trajectory(sd, fx, nf=8):
    """The three golden steps re-run by the CPU oracle in fp64 (same draws, same lr schedule)."""
    T = int(fx["T"])
    _, _, ab = R.make_schedule(T)
    s = {k: (v.double() if v.is_floating_point() else v.clone()) for k, v in sd.items()}
    tr = R.OracleTrainer(s, n_feat=nf, n_cfeat=6, height=64, lr=float(fx["lrate"]))
    x, c = torch.from_numpy(fx["x"]).double(), torch.from_numpy(fx["c"]).double()
    out = []
    for k in range(3):
        w = torch.from_numpy(fx[f"s{k}_sc_w"]).reshape(nf, 1, 1, 1).double()
        b = torch.from_numpy(fx[f"s{k}_sc_b"]).double()
        loss, _, grads = tr.step(x, c, torch.from_numpy(fx[f"s{k}_noise"]).double(), torch.from_numpy(fx[f"s{k}_t"]),
                                 T, ab.double(), (w, b), lr=float(fx[f"s{k}_lr"]))
        out.append((float(loss), {kk: v.detach().clone() for kk, v in tr.sd.items()}, grads))
    return out


def _dev_stats(a, b, keys, unit):
    d = np.concatenate([(np.abs(a[k].double().numpy() - b[k].double().numpy()) / unit).ravel() for k in keys])
    return float(np.sqrt((d ** 2).mean())), float(np.percentile(d, 99)), float(d.max())


def _torch_adam_check(pre, grads, post, m_hip, v_hip, opt, tparams, lr, mprev, vprev):
    """One torch.optim.Adam step on CPU from HIP's pre-step parameters and gradients vs HIP's result."""
    with torch.no_grad():
        for n, p in tparams.items():
            p.copy_(pre[n])
            p.grad = grads[n].clone()
    opt.param_groups[0]["lr"] = lr
    opt.step()
    exact, exact_r, total = 0, 0, 0
    for n, p in tparams.items():
        ref = p.detach().numpy(); got = post[n].numpy()
        st = opt.state[p]
        assert np.array_equal(st["exp_avg"].numpy(), m_hip[n].numpy()), f"{n}: exp_avg differs"
        assert np.array_equal(st["exp_avg_sq"].numpy(), v_hip[n].numpy()), f"{n}: exp_avg_sq differs"
        _ulp_bound(got, ref, pre[n].numpy(), n)
        restated = R.adam_step_restated(pre[n].numpy(), grads[n].numpy(), mprev[n], vprev[n], lr,
                                        opt.state[p]["step"].item())
        exact += int((got == ref).sum()); exact_r += int((got == restated[0]).sum()); total += ref.size
    return exact / total, exact_r / total


def _ulp_bound(got, ref, pre, what):
    """HIP vs this host's torch CPU Adam, a sanity bound only: torch's vectorised CPU sqrt comes from a math library
    whose accuracy depends on the host CPU (17 % of the roots not correctly rounded on the GPU box, 0.6 % in the
    build container, rare elements off by far more than an ulp), so here only |d| <= ulp(p) + 1e-3 |update| is
    asserted.  Exactness is pinned against the restatement (here) and restatement vs torch in the build container
    (tests/test_oracle_adam.py)."""
    upd = np.abs(ref.astype(np.float64) - pre)
    err = np.abs(got.astype(np.float64) - ref)
    bad = err > np.spacing(np.abs(ref)) + upd * 1e-3
    assert not bad.any(), f"{what}: {int(bad.sum())} parameters beyond the ulp bound, e.g. {got[bad][:3]} vs {ref[bad][:3]}"


def _moments(tr):
    m, v = {}, {}
    for n, view in tr.views.items():
        off = view.data_ptr() - tr.flat.data_ptr()
        lo = off // 4
        m[n] = tr.m[lo:lo + view.numel()].view_as(view).cpu().clone()
        v[n] = tr.v[lo:lo + view.numel()].view_as(view).cpu().clone()
    return m, v


@pytest.mark.parametrize("math", ["h3"])
def test_trainer_matches_reference_training_loop(math):
    """Trainer (inject mode, eager) through three reference loop iterations incl. the per-epoch LR decay, under the
    shipped arithmetic h3 (the one bench.py times), every bar on every step.  (Round 4: the x6 / fp32
    parametrisations, which flip one ReLU / MaxPool kink on this golden input in step 0 and needed waivers after it,
    were removed: test_trainer_three_steps_all_arithmetics holds all three arithmetics to the same bars without
    waivers on a kink-free input.)"""
    from cdm_amd import Trainer
    fx = np.load(os.path.join(GOLD, "train_nf8.npz"))
    base = np.load(os.path.join(GOLD, "model_nf8.npz"))
    sd0 = _golden_sd(base, "sd.")
    nf, T, lr0 = 8, int(fx["T"]), float(fx["lrate"])
    m = _model(nf, sd0, math=math)
    x = torch.from_numpy(fx["x"]).cuda(); c = torch.from_numpy(fx["c"]).cuda()
    tr = Trainer(m, lr0, T, x.shape[0], use_graph=False)
    names = list(tr.views)
    tparams = {n: torch.zeros_like(tr.views[n], device="cpu").requires_grad_(True) for n in names}
    opt = torch.optim.Adam(list(tparams.values()), lr=lr0)
    ref64 = _fp64_oracle_trajectory(sd0, fx)
    mprev = {n: np.zeros(tuple(tr.views[n].shape), np.float32) for n in names}
    vprev = {n: np.zeros(tuple(tr.views[n].shape), np.float32) for n in names}
    keep = [n for n in names if not _bn_fed_bias(n)]
    for k in range(3):
        lr = float(fx[f"s{k}_lr"])
        tr.set_lr(lr)
        pre = _params(tr)
        sc = torch.cat([torch.from_numpy(fx[f"s{k}_sc_w"]), torch.from_numpy(fx[f"s{k}_sc_b"])]).cuda()
        inject = (torch.from_numpy(fx[f"s{k}_noise"]).cuda(), torch.from_numpy(fx[f"s{k}_t"]).cuda().int(), sc)
        loss = float(tr.step(x, c, inject=inject).item())
        torch.cuda.synchronize()
        grads = {n: g.detach().cpu().clone() for n, g in tr.grads.items()}
        post = _params(tr)
        mh, vh = _moments(tr)
        # (1) the fused Adam == torch.optim.Adam on identical inputs
        frac, frac_r = _torch_adam_check(pre, grads, post, mh, vh, opt, tparams, lr, mprev, vprev)
        mprev = {n: mh[n].numpy() for n in names}; vprev = {n: vh[n].numpy() for n in names}
        print(f"[{math}] step {k}: Adam bit-identical to the restatement on {100 * frac_r:.4f} %, to this host's "
              f"torch CPU Adam on {100 * frac:.3f} % (rest within the ulp bound)")
        assert frac_r >= 0.99999
        # (2) step-0 gradients vs the fp64 oracle at the criterion of test_train_grads_random_weights_vs_fp64
        #     (per tensor rel L2 <= 1e-2, median <= 5e-3; BN-fed conv biases |g| <= 1e-4 max) — the strict golden bar
        #     is input-dependent under ReLU/MaxPool kink flips; test_train_step_grads_match_reference holds it
        if k == 0:
            g64 = ref64[0][2]
            gmax = max(v.abs().max().item() for v in g64.values())
            errs, errs_ref, names_kept = [], [], []
            for n in names:
                ref = g64[n]
                # analytic-zero gradients: conv biases feeding a BatchNorm, and out.0's bias at n_feat=8 (its
                # GroupNorm(8) has one channel per group): rounding noise only
                if _bn_fed_bias(n) or ref.abs().max().item() <= 1e-6 * gmax:
                    assert grads[n].abs().max().item() <= 1e-4 * gmax, n
                    continue
                errs.append(((grads[n].double() - ref).norm() / ref.norm()).item()); names_kept.append(n)
                errs_ref.append(((torch.from_numpy(fx["s0_grad." + n]).double() - ref).norm() / ref.norm()).item())
            worst = names_kept[int(np.argmax(errs))]
            print(f"[{math}] step-0 grads vs fp64: rel L2 max {max(errs):.2e} ({worst}) median {np.median(errs):.2e} "
                  f"(reference fp32: max {max(errs_ref):.2e} median {np.median(errs_ref):.2e})")
            # a ReLU / MaxPool decision at |z| ~ 1e-6 that flips under a last-bit difference moves the gradients
            # upstream of it by ~1e-2 (test_train_grads_random_weights_vs_fp64): median <= 5e-3, every tensor <= 2e-2
            assert max(errs) <= 2e-2 and float(np.median(errs)) <= 5e-3
        # (3) loss and state after the step vs the reference, anchored on the fp64 oracle
        gold = _golden_sd(fx, f"s{k}_after.")
        loss64, sd64, _ = ref64[k]
        ref_loss_err = abs(float(fx[f"s{k}_loss"]) - loss64)
        # step 0: the reference's own fp32 error (+1e-5 rel); later steps: 1e-4 rel (a ReLU / MaxPool kink flipped in
        # an earlier step's gradient moves the parameters the loss is evaluated at)
        assert abs(loss - loss64) <= 3 * ref_loss_err + (1e-5 if k == 0 else 1e-4) * abs(loss64), \
            (loss, loss64, float(fx[f"s{k}_loss"]))
        got = {n: post[n] for n in names}
        h_rms, h_p99, h_max = _dev_stats(got, sd64, keep, lr0)
        r_rms, r_p99, r_max = _dev_stats(gold, sd64, keep, lr0)
        print(f"[{math}] step {k}: |dp|/lr vs fp64  HIP rms {h_rms:.2e} p99 {h_p99:.2e} max {h_max:.2e} | "
              f"reference fp32 rms {r_rms:.2e} p99 {r_p99:.2e} max {r_max:.2e}")
        _parity.record("trainer_nf8_reference_loop", conv_math=math, step=k, loss=loss, loss_fp64=loss64,
                       loss_err=abs(loss - loss64), loss_err_ref32=ref_loss_err, param_dev_lr_rms=h_rms,
                       param_dev_lr_p99=h_p99, param_dev_lr_rms_ref32=r_rms, param_dev_lr_p99_ref32=r_p99,
                       adam_exact_frac=frac_r)
        assert h_rms <= 3 * r_rms + 1e-3 and h_p99 <= 3 * r_p99 + 1e-3
        for n in names:
            if _bn_fed_bias(n):
                assert (got[n] - gold[n]).abs().max().item() <= 2 * lr0 * (k + 1) + 1e-6, n
        sd_now = {kk: v.detach().cpu() for kk, v in m.state_dict().items()}
        for kk in sd_now:
            if kk.endswith("num_batches_tracked"):
                assert int(sd_now[kk]) == int(gold[kk]) == k + 1, kk
            elif "running" in kk:
                e_h = (sd_now[kk].double() - sd64[kk]).abs().max().item()
                e_r = (gold[kk].double() - sd64[kk]).abs().max().item()
                assert e_h <= 3 * e_r + 1e-5 * sd64[kk].abs().max().item() + 1e-7, (kk, e_h, e_r)


def test_adam_kernel_matches_torch_cpu_adam():
    """cdm_adam on 1,000,003 random parameters (vector bodies + tails), 5 steps with an LR change, against
    torch.optim.Adam on CPU; a DDP-style grad_scale of 1/2 on a summed gradient is checked the same way."""
    import cdm_amd
    from cdm_amd.trainer import adam_bias_table
    L = cdm_amd.lib()
    n = 1_000_003
    g = torch.Generator().manual_seed(3)
    p0 = torch.randn(n, generator=g)
    p = p0.cuda(); m = torch.zeros(n, device="cuda"); v = torch.zeros(n, device="cuda")
    state = torch.tensor([1e-3, 0.0, 0.0, 1.0], dtype=torch.float64, device="cuda")
    bc = adam_bias_table(0.9, 0.999).cuda()
    tp = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([tp], lr=1e-3)
    s = torch.cuda.current_stream().cuda_stream
    mprev, vprev = np.zeros(n, np.float32), np.zeros(n, np.float32)
    for step, lr in enumerate((1e-3, 1e-3, 7.5e-4, 7.5e-4, 3e-4)):
        grad = torch.randn(n, generator=g) * (10.0 ** (step - 2))
        state[0] = lr
        pre = p.cpu()
        gs = (grad * 2).cuda()                        # summed over 2 ranks, scaled by 1/world inside the kernel
        L.cdm_adam(p.data_ptr(), gs.data_ptr(), m.data_ptr(), v.data_ptr(), n, state.data_ptr(), bc.data_ptr(),
                   bc.shape[0], 0.9, 0.999, 1e-8, 0.5, s)
        torch.cuda.synchronize()
        tp.grad = grad.clone()
        opt.param_groups[0]["lr"] = lr
        opt.step()
        ref = tp.detach().numpy(); got = p.cpu().numpy()
        emu = R.adam_step_restated(pre.numpy(), gs.cpu().numpy(), mprev, vprev, lr, step + 1, grad_scale=0.5)
        frac, frac_emu = float((got == ref).mean()), float((got == emu[0]).mean())
        sq_bad = float((torch.sqrt(opt.state[tp]["exp_avg_sq"]).numpy()
                        != np.sqrt(opt.state[tp]["exp_avg_sq"].numpy())).mean())
        print(f"step {step}: {100 * frac_emu:.5f} % bit-identical to the restatement (oracle.adam_step_restated); "
              f"{100 * frac:.4f} % to this host's torch CPU Adam, whose sqrt is not correctly rounded on "
              f"{100 * sq_bad:.3f} % of the elements")
        assert frac_emu >= 0.99999           # (fp64-emulated fma: a double rounding may differ once in ~1e9)
        assert np.array_equal(m.cpu().numpy(), emu[1]) and np.array_equal(v.cpu().numpy(), emu[2])
        _ulp_bound(got, ref, pre.numpy(), f"step {step}")
        mprev, vprev = m.cpu().numpy(), v.cpu().numpy()
        assert np.array_equal(opt.state[tp]["exp_avg"].numpy(), m.cpu().numpy())
        assert np.array_equal(opt.state[tp]["exp_avg_sq"].numpy(), v.cpu().numpy())
        assert float(state[1]) == step + 1


@pytest.mark.parametrize("math", ["h3"])
def test_trainer_graph_replay_equals_eager(math):
    """Same seed, same weights: hipGraph-replayed Trainer == eager Trainer, bit for bit, over 5 Philox-drawn steps
    with an eval-mode forward after step 2 and set_lr before step 4."""
    from cdm_amd import Trainer
    nf, B, T = 16, 4, 1500
    gx = torch.Generator().manual_seed(21)
    x = torch.rand(B, 1, 64, 64, generator=gx).cuda(); c = torch.rand(B, 6, generator=gx).cuda()
    xe = torch.rand(3, 1, 64, 64, generator=gx).cuda(); te = torch.rand(3, generator=gx).cuda()
    runs = []
    for use_graph in (False, True):
        m = _model(nf, seed=5, math=math)
        m.shortcut_source = "device"
        tr = Trainer(m, 1e-3, T, B, seed=9, use_graph=use_graph)
        losses, evals = [], []
        for k in range(5):
            if k == 3:
                tr.set_lr(5e-4)
            losses.append(float(tr.step(x, c).item()))
            if k == 2:
                m.eval()
                m.shortcut_source = "cpu"
                torch.manual_seed(77)
                with torch.no_grad():
                    evals.append(m(xe, te, c[:3]).cpu())
                m.shortcut_source = "device"
                m.train()
        torch.cuda.synchronize()
        assert (tr.graph is not None) == use_graph
        runs.append((tr.flat.cpu(), tr.m.cpu(), tr.v.cpu(), tr.bnflat.cpu(), losses, evals,
                     tr.opt_state.cpu()))
    a, b = runs
    for i, what in enumerate(("params", "exp_avg", "exp_avg_sq", "BN running stats")):
        assert torch.equal(a[i], b[i]), what
    assert a[4] == b[4], "losses"
    assert torch.equal(a[5][0], b[5][0]), "eval forward between steps"
    assert torch.equal(a[6], b[6]) and float(a[6][1]) == 5.0


def test_stage_hooks_fire_after_the_last_write_nf128():
    """Data-parallel correctness without a second GPU: at n_feat=128 / h3 (every fused BN-backward layer live), a
    stream-ordered copy of each stage's gradient slice taken when the engine reports the stage complete (the moment
    the RCCL all-reduce of that slice is enqueued) must equal the final gradient bit for bit — no kernel writes a
    slice after its hook."""
    from cdm_amd import Trainer
    nf, B, T = 128, 2, 1500
    m = _model(nf, seed=8, math="h3")
    m.shortcut_source = "device"
    tr = Trainer(m, 1e-3, T, B, seed=1, use_graph=False)
    seen, snaps = [], {}

    def hook(name):
        lo, hi = tr.ranges[name]
        seen.append(name)
        snaps[name] = tr.gflat[lo:hi].clone()        # on the stream the backward kernels run on

    tr.stage_hook = hook
    g = torch.Generator().manual_seed(4)
    tr.step(torch.rand(B, 1, 64, 64, generator=g).cuda(), torch.rand(B, 6, generator=g).cuda())
    torch.cuda.synchronize()
    assert seen == ["out", "up2", "up1", "up0emb", "down2", "down1", "init"]
    for name, (lo, hi) in tr.ranges.items():
        assert torch.equal(snaps[name], tr.gflat[lo:hi]), f"stage {name} written after its hook"
    assert sum(hi - lo for lo, hi in tr.ranges.values()) == tr.total


def test_global_count_weights_the_gradient():
    """Ragged data-parallel batches: with global_count = 2 B (this rank holds half the samples of the step) the
    gradient is exactly half of the plain step's (power-of-two scale: bit-exact), the loss is unchanged."""
    from cdm_amd import Trainer
    nf, B, T = 16, 3, 1000
    g = torch.Generator().manual_seed(6)
    x = torch.rand(B, 1, 64, 64, generator=g).cuda(); c = torch.rand(B, 6, generator=g).cuda()
    inj = (torch.randn(B, 1, 64, 64, generator=g).cuda(), torch.randint(1, T + 1, (B,), generator=g).int().cuda(),
           (torch.rand(2 * nf, generator=g) * 2 - 1).cuda())
    out = []
    for count in (None, 2 * B):
        m = _model(nf, seed=2, math="h3")
        tr = Trainer(m, 0.0, T, B, use_graph=False)
        loss = float(tr.step(x, c, inject=inj, global_count=count).item())
        out.append((loss, tr.gflat.cpu().clone()))
    assert out[0][0] == out[1][0]
    assert torch.equal(out[0][1] * 0.5, out[1][1])


def test_nonfinite_loss_guard():
    """SURVEY §5 failure guard: a NaN input makes the loss non-finite; the device counter reports it once."""
    from cdm_amd import Trainer
    m = _model(8, seed=1, math="h3")
    m.shortcut_source = "device"
    tr = Trainer(m, 1e-3, 100, 2, use_graph=True)
    x = torch.rand(2, 1, 64, 64, device="cuda"); c = torch.rand(2, 6, device="cuda")
    tr.step(x, c); tr.step(x, c)
    assert tr.check_finite() == 0
    x[0, 0, 3, 5] = float("nan")
    tr.step(x, c)
    assert tr.check_finite() == 1
    assert tr.check_finite() == 0


def trainer_three_steps(math, seed, nf=8, B=4, T=1000, lrs=(1e-3, 1e-3, 7.5e-4)):
    """Three Trainer steps (inject mode) from seeded weights and inputs vs the CPU oracle run in fp32 (the reference's
    arithmetic, bit-exact to it) and in fp64, each run compared on its own branch (tests/_kinks.py): before every step
    HIP's ReLU / MaxPool decisions are read from one engine forward on the step's inputs (BatchNorm state restored) and
    imposed on an fp64 oracle trainer that follows HIP; the reference's fp32 trainer records its own decisions and a
    second fp64 trainer follows those.  Loss and gradients of step k are compared with fp64 evaluated at the run's own
    parameters at the start of step k (so they measure that step's arithmetic, not where Adam's division by the
    near-zero second moments of step 0 left the run); parameters and BN running statistics are compared along the
    trajectories.  Returns per-step metrics (HIP vs its fp64, the reference vs its fp64) and the decisions each flipped
    relative to the other's."""
    from cdm_amd import Trainer
    from _kinks import Kinks, hip_kinks
    torch.manual_seed(100 + seed)
    m = _model(nf, math=math, seed=100 + seed)
    sd0 = R.clone_sd(m.state_dict())
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(B, 1, 64, 64, generator=g); c = torch.rand(B, 6, generator=g)
    draws = [(torch.randn(B, 1, 64, 64, generator=g), torch.randint(1, T + 1, (B,), generator=g),
              torch.rand(2 * nf, generator=g) * 2 - 1) for _ in lrs]
    tr = Trainer(m, lrs[0], T, B, use_graph=False)
    _, _, ab = R.make_schedule(T)
    def oracle(dt):
        s = {k: (v.to(dt) if v.is_floating_point() else v.clone()) for k, v in sd0.items()}
        return R.OracleTrainer(s, n_feat=nf, n_cfeat=6, height=64, lr=lrs[0])
    o32, o64r, o64h = oracle(torch.float32), oracle(torch.float64), oracle(torch.float64)
    names = list(tr.views)
    keep = [n for n in names if not _bn_fed_bias(n)]
    out = []
    for k, (lr, (noise, t, sc)) in enumerate(zip(lrs, draws)):
        # HIP's decisions at this step (its current parameters, the step's perturbed input and shortcut)
        state = {kk: v.detach().clone() for kk, v in m.state_dict().items()}
        xp = R.perturb_input(x, t, noise, ab)
        hk = hip_kinks(m, xp, t / T, c, (sc[:nf].reshape(nf, 1, 1, 1), sc[nf:]), frozen=False)
        m.load_state_dict(state)
        tr.set_lr(lr)
        loss = float(tr.step(x.cuda(), c.cuda(), inject=(noise.cuda(), t.cuda().int(), sc.cuda())).item())
        torch.cuda.synchronize()
        grads = {n: v.detach().cpu().double() for n, v in tr.grads.items()}

        def ostep(otr, dt, kinks):
            w = sc[:nf].reshape(nf, 1, 1, 1).to(dt); b = sc[nf:].to(dt)
            with kinks:
                l, _, gr = otr.step(x.to(dt), c.to(dt), noise.to(dt), t, T, ab.to(dt), (w, b), lr=lr)
            return float(l), gr, {kk: v.detach().clone() for kk, v in otr.sd.items()}

        def at(sd, kinks):
            """loss and gradients of this step in fp64 at the given parameters (a fresh oracle, its Adam unused): the
            step's own arithmetic error, apart from where earlier steps left each run"""
            fresh = R.OracleTrainer({kk: (v.detach().double() if v.is_floating_point() else v.clone())
                                     for kk, v in sd.items()}, n_feat=nf, n_cfeat=6, height=64, lr=0.0)
            l_, g_, _ = ostep(fresh, torch.float64, kinks)
            return l_, g_
        sd32_0 = {kk: v.detach().clone() for kk, v in o32.sd.items()}
        cap = Kinks()
        l32, g32, sd32 = ostep(o32, torch.float32, cap)
        l64, g64r = at(sd32_0, Kinks(cap.relu, cap.pool))
        _, _, sd64r = ostep(o64r, torch.float64, Kinks(cap.relu, cap.pool))
        l64h, g64 = at(state, Kinks(*hk))
        _, _, sd64 = ostep(o64h, torch.float64, Kinks(*hk))
        flips = sum(int((a[0] != b[0]).sum()) for a, b in zip(hk[0], cap.relu)) + \
            sum(int((a != b).sum()) for a, b in zip(hk[1], cap.pool))
        gmax = max(v.abs().max().item() for v in g64.values())
        ge, ge32, worst = [], [], []
        for n in keep:
            if g64[n].abs().max().item() <= 1e-6 * gmax:
                continue
            ge.append(((grads[n] - g64[n]).norm() / g64[n].norm()).item())
            ge32.append(((g32[n].double() - g64r[n]).norm() / g64r[n].norm()).item())
            worst.append((ge[-1], n, ge32[-1]))
        worst.sort(reverse=True)
        print(f"[{math}] seed {seed} step {k}: worst grads (HIP / ref)", [(n, f"{a:.2e}", f"{b:.2e}") for a, n, b in worst[:4]])
        post = _params(tr)
        h = _dev_stats(post, sd64, keep, lrs[0]); r = _dev_stats(sd32, sd64r, keep, lrs[0])
        bn_h = max((v.detach().cpu().double() - sd64[kk]).abs().max().item() for kk, v in m.state_dict().items()
                   if "running" in kk)
        bn_r = max((sd32[kk].double() - sd64r[kk]).abs().max().item() for kk in sd64r if "running" in kk)
        out.append(dict(step=k, flips_vs_ref32=flips, loss_err=abs(loss - l64h), loss_err_ref32=abs(l32 - l64),
                        loss64=l64h,
                        grad_max=max(ge), grad_max_ref32=max(ge32), grad_median=float(np.median(ge)),
                        grad_median_ref32=float(np.median(ge32)), dev_rms=h[0], dev_p99=h[1], dev_rms_ref32=r[0],
                        dev_p99_ref32=r[1], bn_err=bn_h, bn_err_ref32=bn_r))
    return out


@pytest.mark.parametrize("seed", [0, 1, 2])
@pytest.mark.parametrize("math", ["h3", "x6", "fp32"])
def test_trainer_three_steps_all_arithmetics(math, seed):
    """Three Trainer steps under every fp32-class arithmetic on the first three input seeds (round 5: each run on its
    own kink branch, no seed selection — round 4 picked seed 5 of tools/trainer_seed_scan.py), held to the trajectory
    bars without waivers: per step, loss within 3x the reference's own fp32 deviation from fp64 (+1e-6 rel), step
    gradients rel L2 max / median within 3x the reference's (+1e-5), parameters |dp|/lr RMS and p99 within 3x the
    reference's (+1e-3), BN running statistics within 3x the reference's (+1e-6)."""
    res = trainer_three_steps(math, seed)
    for r in res:
        _parity.record("trainer_three_steps_branch", conv_math=math, seed=seed, **r)
        print(f"[{math}] step {r['step']}: loss {r['loss_err']:.2e} (ref {r['loss_err_ref32']:.2e}); grads max "
              f"{r['grad_max']:.2e} (ref {r['grad_max_ref32']:.2e}) median {r['grad_median']:.2e} (ref "
              f"{r['grad_median_ref32']:.2e}); |dp|/lr rms {r['dev_rms']:.2e} (ref {r['dev_rms_ref32']:.2e}) p99 "
              f"{r['dev_p99']:.2e} (ref {r['dev_p99_ref32']:.2e}); BN {r['bn_err']:.2e} (ref {r['bn_err_ref32']:.2e})")
        assert r["loss_err"] <= 3 * r["loss_err_ref32"] + 1e-6 * abs(r["loss64"])
        assert r["grad_max"] <= 3 * r["grad_max_ref32"] + 1e-5
        assert r["grad_median"] <= 3 * r["grad_median_ref32"] + 1e-5
        assert r["dev_rms"] <= 3 * r["dev_rms_ref32"] + 1e-3 and r["dev_p99"] <= 3 * r["dev_p99_ref32"] + 1e-3
        assert r["bn_err"] <= 3 * r["bn_err_ref32"] + 1e-6
