"""Child process of tests/test_gpu_kernels.py::test_deep_staging_bit_exact: runs the bf16 forward halo conv, whose
staging schedule an environment switch selects ($CDM_HALO_DEEP, read once per process by the library), the fused
weight gradients, and the C_in = 1 forward / C_out = 1 input gradient (row or flat-pixel kernels: $CDM_ROW_KERNELS) on
fixed seeded inputs and saves their outputs, so the test can compare two processes bit for bit.  Round 6 adds the
schedule switches $CDM_WGRAD_STAGGER, $CDM_HALO_BEARLY and $CDM_CONVT_DGRAD_MINB (the weight gradient with the producer
BN sums, the h3 halo forward, the h3 ConvT input gradient).

    python tests/_variant_worker.py OUT.pt
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(out_path):
    import cdm_amd
    L = cdm_amd.lib()
    s = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device="cuda").manual_seed(21)
    out = {}
    # one-term forward halo conv with the BN-ReLU staging, several tiles per block and a short last block
    N, H, C = 97, 64, 128
    P = N * H * H
    x = torch.randn(P, C, device="cuda", generator=g)
    ps, pt = torch.rand(C, device="cuda", generator=g) + 0.5, torch.randn(C, device="cuda", generator=g) * 0.3
    W = torch.randn(C, C, 3, 3, device="cuda", generator=g) * 0.05
    b = torch.randn(C, device="cuda", generator=g)
    wpk = torch.empty(9 * C, C, device="cuda")
    L.cdm_pack_conv3x3(W.data_ptr(), b.data_ptr(), C, C, None, None, None, None, 0.0, wpk.data_ptr(), None, None, 16, s)
    wx = torch.empty(9 * C // 16 * 3 * C * 16, dtype=torch.bfloat16, device="cuda")
    L.cdm_split_bf16x3(wpk.data_ptr(), C, 9 * C, C, wx.data_ptr(), s)
    y = torch.empty(P, C, device="cuda")
    st = torch.empty(P // 128, 2, C, device="cuda")
    assert L.cdm_conv3x3_fwd_x16_ex(x.data_ptr(), N, H, H, C, C, ps.data_ptr(), pt.data_ptr(), wx.data_ptr(), None,
                                    None, b.data_ptr(), y.data_ptr(), C, C, 0, st.data_ptr(), C, 16, None, None, 0, 1,
                                    0, s) == 0
    out["halo_y"], out["halo_stats"] = y.cpu(), st.cpu()
    # kernel-row weight gradient, BN-backward dY staging + BN-ReLU X staging, both 16-bit arithmetics
    from cdm_amd.engine import wgrad_splits
    for nterm in (4, 1):
        for (B, S, ci, co) in ((4, 64, 128, 128), (3, 32, 256, 256)):
            P = B * S * S
            gy = torch.randn(P, co, device="cuda", generator=g) * 1e-2
            yy = torch.randn(P, co, device="cuda", generator=g)
            xx = torch.randn(P, ci, device="cuda", generator=g)
            cf = [torch.randn(co, device="cuda", generator=g) for _ in range(7)]
            cf[3] = cf[3].abs() + 0.1
            xs_, xt_ = torch.rand(ci, device="cuda", generator=g) + 0.5, torch.randn(ci, device="cuda", generator=g)
            am = torch.ones(2, device="cuda") * 8.0
            sp = wgrad_splits(P, co, 9 * ci)
            slab = torch.empty(sp * co * 9 * ci, device="cuda")
            assert L.cdm_conv3x3_wgrad_x16_ex(gy.data_ptr(), co, yy.data_ptr(), co, *[t.data_ptr() for t in cf], co,
                                              xx.data_ptr(), B, S, S, ci, ci, xs_.data_ptr(), xt_.data_ptr(), None, 0,
                                              None, None, None, am.data_ptr(), am.data_ptr() + 4, sp, slab.data_ptr(),
                                              nterm, 0, s) == 0
            out[f"wgrad_{nterm}_{S}"] = slab.cpu()
    # round 6 schedules: the row weight gradient with the producer BN sums (64-pixel K steps under h3 at 64^2; staggered
    # look-ahead order vs lock-step, $CDM_WGRAD_STAGGER), the h3 halo forward (B one kernel row earlier,
    # $CDM_HALO_BEARLY), the h3 ConvT 2x2 input gradient (two vs three blocks per CU, $CDM_CONVT_DGRAD_MINB)
    for nterm in (4, 1):
        B, S, ci, co = 4, 64, 128, 128
        P = B * S * S
        yx = torch.randn(P, ci, device="cuda", generator=g)
        gx = torch.randn(P, ci, device="cuda", generator=g)
        dyy = torch.randn(P, co, device="cuda", generator=g) * 1e-2
        xs_, xt_ = torch.rand(ci, device="cuda", generator=g) + 0.5, torch.randn(ci, device="cuda", generator=g) * 0.1
        mu, inv = torch.randn(ci, device="cuda", generator=g) * 0.1, torch.rand(ci, device="cuda", generator=g) + 0.5
        am = torch.ones(4, device="cuda") * 8.0
        sp = wgrad_splits(P, co, 9 * ci)
        slab = torch.empty(sp * co * 9 * ci, device="cuda")
        sums = torch.empty(sp * 3 * (co // 128) * 5 * ci, device="cuda")
        assert L.cdm_conv3x3_wgrad_x16_ex(dyy.data_ptr(), co, None, 0, None, None, None, None, None, None, None, co,
                                          yx.data_ptr(), B, S, S, ci, ci, xs_.data_ptr(), xt_.data_ptr(), gx.data_ptr(),
                                          ci, mu.data_ptr(), inv.data_ptr(), sums.data_ptr(), am.data_ptr(),
                                          am.data_ptr() + 4, sp, slab.data_ptr(), nterm, 0, s) == 0
        out[f"wgrad_sums_{nterm}"], out[f"wgrad_sums_sums_{nterm}"] = slab.cpu(), sums.cpu()
    N, H, C = 5, 64, 128
    P = N * H * H
    xh = torch.randn(P, C, device="cuda", generator=g).relu()
    wpk = torch.empty(9 * C, C, device="cuda")
    Wh, bh = torch.randn(C, C, 3, 3, device="cuda", generator=g) * 0.05, torch.randn(C, device="cuda", generator=g)
    L.cdm_pack_conv3x3(Wh.data_ptr(), bh.data_ptr(), C, C, None, None, None, None, 0.0, wpk.data_ptr(), None, None, 16, s)
    amh = torch.zeros(2, device="cuda")
    L.cdm_amax_f32(wpk.data_ptr(), 9 * C, C, C, amh.data_ptr() + 4, 0, s)
    L.cdm_amax_f32(xh.data_ptr(), P, C, C, amh.data_ptr(), 0, s)
    wxh = torch.empty(9 * C // 16 * 3 * C * 16, dtype=torch.bfloat16, device="cuda")
    L.cdm_split_f16x2(wpk.data_ptr(), C, 9 * C, C, amh.data_ptr() + 4, wxh.data_ptr(), s)
    yh, sth = torch.empty(P, C, device="cuda"), torch.empty((P + 127) // 128, 2, C, device="cuda")
    assert L.cdm_conv3x3_fwd_h3(xh.data_ptr(), N, H, H, C, C, wxh.data_ptr(), amh.data_ptr(), amh.data_ptr() + 4, None,
                                yh.data_ptr(), C, C, 0, sth.data_ptr(), C, 16, None, s) == 0
    out["halo_h3_y"], out["halo_h3_stats"] = yh.cpu(), sth.cpu()
    N, H, Co, Ci = 2, 32, 128, 256                       # ConvT input grid H x H, its output channels Co
    dyt = torch.randn(N * 4 * H * H, Co, device="cuda", generator=g)
    wt = torch.randn(4 * Co, Ci, device="cuda", generator=g) * 0.05
    amt = torch.zeros(2, device="cuda")
    L.cdm_amax_f32(dyt.data_ptr(), N * 4 * H * H, Co, Co, amt.data_ptr(), 0, s)
    L.cdm_amax_f32(wt.data_ptr(), 4 * Co, Ci, Ci, amt.data_ptr() + 4, 0, s)
    wxt = torch.empty(4 * Co // 16 * 3 * Ci * 16, dtype=torch.bfloat16, device="cuda")
    L.cdm_split_f16x2(wt.data_ptr(), Ci, 4 * Co, Ci, amt.data_ptr() + 4, wxt.data_ptr(), s)
    dxt = torch.empty(N * H * H, Ci, device="cuda")
    assert L.cdm_convT2x2_dgrad_x16(dyt.data_ptr(), N, H, H, Co, Co, wxt.data_ptr(), amt.data_ptr(),
                                    amt.data_ptr() + 4, dxt.data_ptr(), Ci, Ci, 0, 4, s) == 0
    out["convT_dgrad_h3"] = dxt.cpu()
    # C_in = 1 forward and C_out = 1 input gradient: the row kernels vs the flat-pixel kernels ($CDM_ROW_KERNELS)
    for (N, H, W, C) in ((3, 64, 64, 128), (2, 32, 32, 256), (2, 24, 40, 64), (1, 256, 256, 128)):
        x1 = torch.randn(N * H * W, device="cuda", generator=g)
        w9 = torch.randn(9 * C, device="cuda", generator=g) * 0.3
        b1 = torch.randn(C, device="cuda", generator=g)
        for relu in (0, 1):
            y1 = torch.empty(N * H * W, C, device="cuda")
            am = torch.zeros(1, device="cuda")
            assert L.cdm_conv3x3_cin1_fwd(x1.data_ptr(), N, H, W, w9.data_ptr(), b1.data_ptr(), y1.data_ptr(), C, C,
                                          relu, am.data_ptr(), s) == 0
            out[f"cin1_{N}_{H}_{W}_{C}_{relu}"], out[f"cin1_amax_{N}_{H}_{W}_{C}_{relu}"] = y1.cpu(), am.cpu()
        dz = torch.empty(N * H * W, C + 4, device="cuda")   # ld > C
        assert L.cdm_conv3x3_cout1_dgrad(x1.data_ptr(), N, H, W, C, w9.data_ptr(), dz.data_ptr(), C + 4, s) == 0
        out[f"cout1_dgrad_{N}_{H}_{W}_{C}"] = dz[:, :C].cpu()
    torch.cuda.synchronize()
    torch.save(out, out_path)


if __name__ == "__main__":
    main(sys.argv[1])
