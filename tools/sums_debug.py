"""Producer BN-backward sums in the consumer weight gradient (PreBnReluSums): kernel-level check against the
cdm_norm_bwd_reduce mode-0 slab, and model-level per-tensor gradient differences sums on / off (GPU box).

    python tools/sums_debug.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def kernel_check(B, S, cin, cout, nterm):
    import cdm_amd
    from cdm_amd.engine import wgrad_splits
    L = cdm_amd.lib()
    st = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device="cuda").manual_seed(5)
    P = B * S * S
    y = torch.randn(P, cin, device="cuda", generator=g)          # producer pre-norm output (the X operand)
    gx = torch.randn(P, cin, device="cuda", generator=g)         # grad wrt relu(y s + t)
    dy = torch.randn(P, cout, device="cuda", generator=g) * 1e-2
    s_ = torch.rand(cin, device="cuda", generator=g) + 0.5
    t_ = torch.randn(cin, device="cuda", generator=g) * 0.1
    mean = torch.randn(cin, device="cuda", generator=g) * 0.1
    inv = torch.rand(cin, device="cuda", generator=g) + 0.5
    am = torch.ones(4, device="cuda") * 8.0
    sp = wgrad_splits(P, cout, 9 * cin)
    slab = torch.empty(sp * cout * 9 * cin, device="cuda")
    sums = torch.full((sp * 5 * cin,), float("nan"), device="cuda")
    rc = L.raw("cdm_conv3x3_wgrad_x16_ex")(dy.data_ptr(), cout, None, 0, None, None, None, None, None, None, None, cout,
                                           y.data_ptr(), B, S, S, cin, cin, s_.data_ptr(), t_.data_ptr(),
                                           gx.data_ptr(), cin, mean.data_ptr(), inv.data_ptr(), sums.data_ptr(),
                                           am.data_ptr(), am.data_ptr() + 4, sp, slab.data_ptr(), nterm, st)
    torch.cuda.synchronize()
    got = sums.view(sp, 5, cin).double().sum(0)
    zp = y * s_ + t_
    gp = torch.where(zp > 0, gx, torch.zeros_like(gx)).double()
    xh = ((y - mean) * inv).double()
    ref = torch.stack([gp.sum(0), (gp * xh).sum(0), xh.sum(0)])
    g3 = torch.stack([got[0], got[1], got[4]])
    nan = int(torch.isnan(sums.view(sp, 5, cin)).sum())
    err = ((g3 - ref).abs().max(dim=1).values / ref.abs().max(dim=1).values).tolist()
    print(f"kernel B={B} S={S} {cin}->{cout} nterm={nterm} rc={rc} splits={sp} nan={nan} rel err S1/S2/S5 = "
          f"{[f'{e:.2e}' for e in err]}", flush=True)


def model_check(math, B=3):
    import cdm_amd.model as M
    from oracle import ref_cpu as R
    nf, T = 128, 1500
    g = torch.Generator().manual_seed(17)
    x = torch.rand(B, 1, 64, 64, generator=g); noise = torch.randn(B, 1, 64, 64, generator=g)
    c = torch.rand(B, 6, generator=g); tt = torch.randint(1, T + 1, (B,), generator=g)
    _, _, ab = R.make_schedule(T)
    xp = R.perturb_input(x, tt, noise, ab)
    eng = M.get_engine(nf, 6, 64, torch.device("cuda", 0), math)
    out = []
    for on in (True, False):
        eng.fuse_bn_sums = on
        M._WS.clear()
        torch.manual_seed(18)
        m = M.ContextUnet(1, nf, 6, 64, conv_math=math).cuda().train()
        torch.manual_seed(36)
        pred = m(xp.cuda(), (tt / T).cuda(), c.cuda())
        F.mse_loss(pred, noise.cuda()).backward()
        out.append({k: p.grad.detach().double().cpu() for k, p in m.named_parameters()})
    eng.fuse_bn_sums = True
    M._WS.clear()
    rows = []
    for k, ref in out[1].items():
        if ref.norm() == 0:
            continue
        rows.append((((out[0][k] - ref).norm() / ref.norm()).item(), k))
    rows.sort()
    print(f"model [{math}] sums on vs off, worst 12:", flush=True)
    for e, k in rows[-12:]:
        print(f"   {e:.3e}  {k}", flush=True)


if __name__ == "__main__":
    for nterm in (4, 1):
        for shp in ((2, 64, 128, 128), (2, 32, 256, 256), (2, 32, 128, 256), (3, 32, 128, 128)):
            kernel_check(*shp, nterm)
    for math in ("h3", "bf16"):
        model_check(math)
