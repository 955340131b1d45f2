"""Op-level parity of the HIP contraction kernels against plain torch fp32 on CPU (GPU box only).

Tolerance: fp32 MFMA vs CPU fp32 with different summation order -> |err| <= 2e-5 * max|ref| + 1e-5.
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def L():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import cdm_amd
    return cdm_amd.lib()


def _s():
    return torch.cuda.current_stream().cuda_stream


def _close(got, ref, tol=2e-5):
    got = got.detach().float().cpu(); ref = ref.detach().float().cpu()
    err = (got - ref).abs().max().item()
    bound = tol * ref.abs().max().item() + 1e-5
    assert err <= bound, f"max err {err:.3e} > {bound:.3e}"


def _nhwc(x):  # NCHW cpu -> NHWC cuda
    return x.permute(0, 2, 3, 1).contiguous().cuda()


def _nchw(y, N, H, W, C):
    return y.reshape(N, H, W, C).permute(0, 3, 1, 2).cpu()


def _pack3x3(L, W, b, kc=0):
    Cout, Cin = W.shape[:2]
    wpk = torch.empty(9 * Cin, Cout, device="cuda"); wdg = torch.empty(9 * Cout, Cin, device="cuda")
    L.cdm_pack_conv3x3(W.data_ptr(), b.data_ptr(), Cin, Cout, None, None, None, None, 0.0, wpk.data_ptr(), None,
                       wdg.data_ptr(), kc, _s())
    return wpk, wdg


@pytest.mark.parametrize("kc", [0, 16])
@pytest.mark.parametrize("N,H,Cin,Cout", [(2, 16, 32, 64), (1, 64, 128, 128), (3, 8, 8, 16), (2, 32, 256, 128)])
def test_conv3x3_fwd_dgrad_wgrad(L, N, H, Cin, Cout, kc):
    if kc and (Cin % kc or Cout % kc):
        pytest.skip("chunked K needs channels % 16 == 0")
    torch.manual_seed(0)
    x = torch.randn(N, Cin, H, H); W = torch.randn(Cout, Cin, 3, 3) * 0.1; b = torch.randn(Cout)
    gy = torch.randn(N, Cout, H, H)
    xg, Wg, bg = x.clone().requires_grad_(), W.clone().requires_grad_(), b.clone()
    ref = F.conv2d(xg, Wg, bg, padding=1)
    ref.backward(gy)
    Wc, bc = W.cuda(), b.cuda()
    wpk, wdg = _pack3x3(L, Wc, bc, kc)
    xn = _nhwc(x)
    y = torch.empty(N * H * H, Cout, device="cuda")
    ntile = (N * H * H + 127) // 128
    stats = torch.zeros(ntile, 2, Cout, device="cuda")
    L.cdm_conv3x3_fwd(xn.data_ptr(), N, H, H, Cin, Cin, wpk.data_ptr(), bc.data_ptr(), y.data_ptr(), Cout, Cout, 0,
                      stats.data_ptr(), Cout, kc, _s())
    torch.cuda.synchronize()
    _close(_nchw(y, N, H, H, Cout), ref.detach())
    ysum = ref.detach().permute(0, 2, 3, 1).reshape(-1, Cout)
    _close(stats[:, 0].sum(0), ysum.sum(0), 1e-4)
    _close(stats[:, 1].sum(0), (ysum ** 2).sum(0), 1e-4)
    # dgrad = conv with flipped / transposed weights
    gyn = _nhwc(gy)
    dx = torch.empty(N * H * H, Cin, device="cuda")
    L.cdm_conv3x3_fwd(gyn.data_ptr(), N, H, H, Cout, Cout, wdg.data_ptr(), None, dx.data_ptr(), Cin, Cin, 0, None, 0,
                      kc, _s())
    torch.cuda.synchronize()
    _close(_nchw(dx, N, H, H, Cin), xg.grad)
    # wgrad (split-K slabs) + reduce into OIHW
    for splits in (1, 7):
        sp = L.raw("cdm_gemm_splits")(N * H * H, splits)
        slab = torch.empty(sp, Cout, 9 * Cin, device="cuda")
        L.cdm_conv3x3_wgrad(gyn.data_ptr(), Cout, Cout, xn.data_ptr(), N, H, H, Cin, Cin, sp, slab.data_ptr(), _s())
        dW = torch.empty(Cout, Cin, 3, 3, device="cuda")
        L.cdm_slab_reduce(slab.data_ptr(), sp, Cout, 9 * Cin, dW.data_ptr(), 9 * Cin, 1, 9, Cin, 0, 1.0, _s())
        torch.cuda.synchronize()
        _close(dW, Wg.grad, 5e-5)


def test_conv3x3_channel_slices(L):
    """read from / write into channel slices of wider NHWC buffers (the torch.cat elimination)."""
    torch.manual_seed(1)
    N, H, Cin, Cout = 2, 16, 32, 32
    big = torch.randn(N, H, H, 3 * Cin, device="cuda")
    x = big[..., Cin:2 * Cin]
    W = torch.randn(Cout, Cin, 3, 3, device="cuda") * 0.1; b = torch.randn(Cout, device="cuda")
    wpk, _ = _pack3x3(L, W, b, 16)
    out = torch.zeros(N, H, H, 2 * Cout, device="cuda")
    L.cdm_conv3x3_fwd(big.data_ptr() + 4 * Cin, N, H, H, Cin, 3 * Cin, wpk.data_ptr(), b.data_ptr(),
                      out.data_ptr() + 4 * Cout, 2 * Cout, Cout, 1, None, 0, 16, _s())
    torch.cuda.synchronize()
    ref = F.relu(F.conv2d(x.permute(0, 3, 1, 2).cpu(), W.cpu(), b.cpu(), padding=1)).permute(0, 2, 3, 1)
    _close(out[..., Cout:], ref)
    assert out[..., :Cout].abs().max().item() == 0.0


@pytest.mark.parametrize("N,Hin,Cin,Cout", [(2, 8, 64, 32), (1, 16, 512, 128), (3, 4, 16, 8), (2, 32, 256, 128)])
def test_convT2x2(L, N, Hin, Cin, Cout):
    torch.manual_seed(2)
    x = torch.randn(N, Cin, Hin, Hin); W = torch.randn(Cin, Cout, 2, 2) * 0.1; b = torch.randn(Cout)
    gy = torch.randn(N, Cout, 2 * Hin, 2 * Hin)
    xg, Wg = x.clone().requires_grad_(), W.clone().requires_grad_()
    ref = F.conv_transpose2d(xg, Wg, b, stride=2)
    ref.backward(gy)
    Wc = W.cuda(); bc = b.cuda()
    wt = torch.empty(Cin, 4 * Cout, device="cuda"); wtT = torch.empty(4 * Cout, Cin, device="cuda")
    L.cdm_pack_convT(Wc.data_ptr(), Cin, Cout, 4, wt.data_ptr(), wtT.data_ptr(), _s())
    xn = _nhwc(x)
    y = torch.empty(N * 4 * Hin * Hin, Cout, device="cuda")
    am = torch.zeros(1, device="cuda")
    L.cdm_convT2x2_fwd(xn.data_ptr(), N, Hin, Hin, Cin, Cin, wt.data_ptr(), bc.data_ptr(), y.data_ptr(), Cout, Cout,
                       am.data_ptr(), _s())
    torch.cuda.synchronize()
    _close(_nchw(y, N, 2 * Hin, 2 * Hin, Cout), ref.detach())
    assert am.item() == y.abs().max().item()          # fused producer max (h3 operand scale)
    # h3 forward (scaled fp16 hi/lo split on the matrix cores): same fp32 tolerance, fused max|y|
    wx, amw = _split_h3(L, wt, Cin, 4 * Cout)
    amx = _amax(L, xn, N * Hin * Hin, Cin)
    y3 = torch.empty_like(y)
    am3 = torch.zeros(1, device="cuda")
    L.cdm_convT2x2_fwd_h3(xn.data_ptr(), N, Hin, Hin, Cin, Cin, wx.data_ptr(), amx.data_ptr(), amw.data_ptr(),
                          bc.data_ptr(), y3.data_ptr(), Cout, Cout, am3.data_ptr(), _s())
    torch.cuda.synchronize()
    _close(_nchw(y3, N, 2 * Hin, 2 * Hin, Cout), ref.detach())
    assert am3.item() == y3.abs().max().item()
    # the two-deep prefetch kernel (default where M, 4 Cout % 128 == 0 and Cin % 32 == 0) against gemm_x3: the same
    # products in the same order, bit for bit — h3 and the one-term bf16 form
    wxb = torch.empty((Cin + 15) // 16 * 3 * 4 * Cout * 16, dtype=torch.bfloat16, device="cuda")
    L.cdm_split_bf16x3(wt.data_ptr(), 4 * Cout, Cin, 4 * Cout, wxb.data_ptr(), _s())
    outs = {}
    for deep in ("1", "0"):
        os.environ["CDM_CONVT_DEEP"] = deep
        try:
            for nterm, w_, aw in ((4, wx, amw), (1, wxb, None)):
                o = torch.empty_like(y); ao = torch.zeros(1, device="cuda")
                L.cdm_convT2x2_fwd_x16(xn.data_ptr(), N, Hin, Hin, Cin, Cin, w_.data_ptr(),
                                       amx.data_ptr() if aw is not None else None,
                                       aw.data_ptr() if aw is not None else None, bc.data_ptr(), o.data_ptr(), Cout,
                                       Cout, ao.data_ptr(), nterm, _s())
                torch.cuda.synchronize()
                outs[deep, nterm] = (o, ao)
        finally:
            del os.environ["CDM_CONVT_DEEP"]
    for nterm in (4, 1):
        assert torch.equal(outs["1", nterm][0], outs["0", nterm][0]) and torch.equal(outs["1", nterm][1],
                                                                                     outs["0", nterm][1])
    assert torch.equal(outs["1", 4][0], y3)
    _close(_nchw(outs["1", 1][0], N, 2 * Hin, 2 * Hin, Cout), ref.detach(), 2e-2)
    gyn = _nhwc(gy)
    dx = torch.empty(N * Hin * Hin, Cin, device="cuda")
    L.cdm_convT2x2_dgrad(gyn.data_ptr(), N, Hin, Hin, Cout, Cout, wtT.data_ptr(), dx.data_ptr(), Cin, Cin, 0, _s())
    torch.cuda.synchronize()
    _close(_nchw(dx, N, Hin, Hin, Cin), xg.grad)
    sp = L.raw("cdm_gemm_splits")(N * Hin * Hin, 3)
    slab = torch.empty(sp, Cin, 4 * Cout, device="cuda")
    L.cdm_convT2x2_wgrad(xn.data_ptr(), N, Hin, Hin, Cin, Cin, gyn.data_ptr(), Cout, Cout, sp, slab.data_ptr(), _s())
    dW = torch.empty(Cin, Cout, 2, 2, device="cuda")
    L.cdm_slab_reduce(slab.data_ptr(), sp, Cin, 4 * Cout, dW.data_ptr(), 4 * Cout, 1, 4, Cout, 0, 1.0, _s())
    torch.cuda.synchronize()
    _close(dW, Wg.grad, 5e-5)
    # h3 backward (engine default): dgrad from the pre-split wpkT, wgrad with both operands scaled + split
    amg = _amax(L, gyn, N * 4 * Hin * Hin, Cout)
    wxT, amwT = _split_h3(L, wtT, 4 * Cout, Cin)
    dx3 = torch.empty_like(dx)
    L.cdm_convT2x2_dgrad_h3(gyn.data_ptr(), N, Hin, Hin, Cout, Cout, wxT.data_ptr(), amg.data_ptr(), amwT.data_ptr(),
                            dx3.data_ptr(), Cin, Cin, 0, _s())
    torch.cuda.synchronize()
    _close(_nchw(dx3, N, Hin, Hin, Cin), xg.grad)
    # the input gradient on the two-deep prefetch GEMM vs gemm_x3, bit for bit (plain and accumulating epilogue)
    base = torch.randn_like(dx)
    got = {}
    for deep in ("1", "0"):
        os.environ["CDM_CONVT_DEEP"] = deep
        try:
            for flags in (0, 2):
                o = base.clone()
                L.cdm_convT2x2_dgrad_h3(gyn.data_ptr(), N, Hin, Hin, Cout, Cout, wxT.data_ptr(), amg.data_ptr(),
                                        amwT.data_ptr(), o.data_ptr(), Cin, Cin, flags, _s())
                torch.cuda.synchronize()
                got[deep, flags] = o
        finally:
            del os.environ["CDM_CONVT_DEEP"]
    for flags in (0, 2):
        assert torch.equal(got["1", flags], got["0", flags])
    assert torch.equal(got["1", 0], dx3)
    if Hin % 8 == 0:
        slab.fill_(float("nan"))
        L.cdm_convT2x2_wgrad_h3(xn.data_ptr(), N, Hin, Hin, Cin, Cin, gyn.data_ptr(), Cout, Cout, amx.data_ptr(),
                                amg.data_ptr(), sp, slab.data_ptr(), _s())
        dW3 = torch.empty_like(dW)
        L.cdm_slab_reduce(slab.data_ptr(), sp, Cin, 4 * Cout, dW3.data_ptr(), 4 * Cout, 1, 4, Cout, 0, 1.0, _s())
        torch.cuda.synchronize()
        _close(dW3, Wg.grad, 5e-5)


@pytest.mark.parametrize("M,K,N,splits", [(5, 256, 4096, 1), (256, 256, 8192, 1), (10, 4096, 64, 16), (130, 36, 132, 1)])
def test_gemm_and_tn(L, M, K, N, splits):
    torch.manual_seed(3)
    a = torch.randn(M, K); b = torch.randn(K, N); bias = torch.randn(64)
    ref = a @ b + bias.repeat(N // 64 + 1)[:N] if N % 64 == 0 else a @ b
    ac, bc = a.cuda(), b.cuda()
    c = torch.empty(M, N, device="cuda")
    sp = L.raw("cdm_gemm_splits")(K, splits)
    slab = torch.empty(max(sp, 1), M, N, device="cuda")
    use_bias = N % 64 == 0 and sp == 1
    L.cdm_gemm_f32(ac.data_ptr(), K, M, K, bc.data_ptr(), N, N, c.data_ptr(), N,
                   bias.cuda().data_ptr() if use_bias else None, 64, 0, sp, slab.data_ptr(), _s())
    if sp > 1:
        L.cdm_slab_reduce(slab.data_ptr(), sp, M, N, c.data_ptr(), N, 0, 1, N, 0, 1.0, _s())
    torch.cuda.synchronize()
    _close(c, ref if use_bias else a @ b, 5e-5)
    # A^T B
    at = torch.randn(K, M if M % 4 == 0 else 4 * ((M + 3) // 4))
    Mt = at.shape[1]
    reft = at.t() @ b
    slab = torch.empty(3, Mt, N, device="cuda")
    sp = L.raw("cdm_gemm_splits")(K, 3)
    L.cdm_gemm_tn_f32(at.cuda().data_ptr(), Mt, Mt, K, bc.data_ptr(), N, N, sp, slab.data_ptr(), _s())
    out = torch.empty(Mt, N, device="cuda")
    L.cdm_slab_reduce(slab.data_ptr(), sp, Mt, N, out.data_ptr(), N, 0, 1, N, 0, 1.0, _s())
    torch.cuda.synchronize()
    _close(out, reft, 5e-5)


@pytest.mark.parametrize("nterm,tol", [(6, 2e-5), (3, 2e-4), (1, 2e-2)])
@pytest.mark.parametrize("N,H,Cin,Cout,kc", [(2, 16, 32, 64, 16), (1, 64, 128, 128, 16), (3, 8, 8, 16, 0),
                                              (2, 32, 256, 128, 16), (1, 8, 12, 20, 0)])
def test_conv3x3_split_bf16(L, N, H, Cin, Cout, kc, nterm, tol):
    """cdm_conv3x3_fwd_x3 (split-bf16 MFMA) fwd + dgrad + stats against torch fp32 conv."""
    torch.manual_seed(4)
    x = torch.randn(N, Cin, H, H); W = torch.randn(Cout, Cin, 3, 3) * 0.1; b = torch.randn(Cout)
    gy = torch.randn(N, Cout, H, H)
    xg, Wg = x.clone().requires_grad_(), W.clone().requires_grad_()
    ref = F.conv2d(xg, Wg, b, padding=1)
    ref.backward(gy)
    Wc, bc = W.cuda(), b.cuda()
    wpk, wdg = _pack3x3(L, Wc, bc, kc)
    split = lambda w, K, NN: _split(L, w, K, NN)
    wx, wdx = split(wpk, 9 * Cin, Cout), split(wdg, 9 * Cout, Cin)
    y = torch.empty(N * H * H, Cout, device="cuda")
    stats = torch.zeros((N * H * H + 127) // 128, 2, Cout, device="cuda")
    xn0, gyn0 = _nhwc(x), _nhwc(gy)
    L.cdm_conv3x3_fwd_x3(xn0.data_ptr(), N, H, H, Cin, Cin, wx.data_ptr(), bc.data_ptr(), y.data_ptr(), Cout,
                         Cout, 0, stats.data_ptr(), Cout, kc, nterm, _s())
    dx = torch.empty(N * H * H, Cin, device="cuda")
    L.cdm_conv3x3_fwd_x3(gyn0.data_ptr(), N, H, H, Cout, Cout, wdx.data_ptr(), None, dx.data_ptr(), Cin, Cin, 0,
                         None, 0, kc, nterm, _s())
    torch.cuda.synchronize()
    _close(_nchw(y, N, H, H, Cout), ref.detach(), tol)
    _close(_nchw(dx, N, H, H, Cin), xg.grad, tol)
    ysum = ref.detach().permute(0, 2, 3, 1).reshape(-1, Cout)
    _close(stats[:, 0].sum(0), ysum.sum(0), max(tol, 1e-4))
    gyn, xn = _nhwc(gy), _nhwc(x)   # keep both alive: the launch is asynchronous
    for splits in (1, 7):   # weight gradient, split-K slabs
        sp = L.raw("cdm_gemm_splits")(N * H * H, splits)
        slab = torch.empty(sp, Cout, 9 * Cin, device="cuda")
        L.cdm_conv3x3_wgrad_x3(gyn.data_ptr(), Cout, Cout, xn.data_ptr(), N, H, H, Cin, Cin, sp, slab.data_ptr(),
                               nterm, _s())
        dW = torch.empty(Cout, Cin, 3, 3, device="cuda")
        L.cdm_slab_reduce(slab.data_ptr(), sp, Cout, 9 * Cin, dW.data_ptr(), 9 * Cin, 1, 9, Cin, 0, 1.0, _s())
        torch.cuda.synchronize()
        _close(dW, Wg.grad, max(tol, 5e-5))


def _split(L, w, K, NN):
    out = torch.empty(((K + 15) // 16) * 3 * NN * 16, dtype=torch.bfloat16, device="cuda")
    L.cdm_split_bf16x3(w.data_ptr(), NN, K, NN, out.data_ptr(), _s())
    return out


def test_split_bf16x3_terms_sum_to_fp32(L):
    """hi + mid + lo reproduces every fp32 weight to <= 2^-24 relative; layout [K/16][3][N][16]."""
    torch.manual_seed(5)
    K, NN = 40, 12
    w = (torch.randn(K, NN) * torch.logspace(-3, 3, K)[:, None]).cuda()
    xs = _split(L, w, K, NN).float().reshape(-1, 3, NN, 16)          # [kt][term][n][kk]
    rec = xs.double().sum(1).permute(0, 2, 1).reshape(-1, NN)[:K]   # [k][n]
    err = ((rec - w.double()).abs() / w.double().abs()).max().item()
    assert err <= 2.0 ** -24, err
    assert xs.reshape(-1, 3, NN, 16).permute(0, 3, 1, 2).reshape(-1, 3, NN)[K:].abs().max().item() == 0.0


def _split_h3(L, w, K, NN):
    am = torch.empty(1, device="cuda")
    L.cdm_amax_f32(w.data_ptr(), K, NN, NN, am.data_ptr(), 0, _s())
    out = torch.empty(((K + 15) // 16) * 3 * NN * 16, dtype=torch.bfloat16, device="cuda")
    L.cdm_split_f16x2(w.data_ptr(), NN, K, NN, am.data_ptr(), out.data_ptr(), _s())
    return out, am


def _amax(L, t, rows, C):
    am = torch.empty(1, device="cuda")
    L.cdm_amax_f32(t.data_ptr(), rows, C, C, am.data_ptr(), 0, _s())
    return am


def _conv_h3(L, x, W, b, gy, kc):
    """fwd, dgrad (NCHW) and wgrad (OIHW) of the h3 conv path for CPU inputs."""
    N, Cin, H, _ = x.shape
    Cout = W.shape[0]
    Wc, bc = W.cuda(), b.cuda()
    wpk, wdg = _pack3x3(L, Wc, bc, kc)
    (wx, amw), (wdx, amd) = _split_h3(L, wpk, 9 * Cin, Cout), _split_h3(L, wdg, 9 * Cout, Cin)
    xn, gyn = _nhwc(x), _nhwc(gy)
    amx, amg = _amax(L, xn, N * H * H, Cin), _amax(L, gyn, N * H * H, Cout)
    y = torch.empty(N * H * H, Cout, device="cuda")
    amy = torch.zeros(1, device="cuda")
    L.cdm_conv3x3_fwd_h3(xn.data_ptr(), N, H, H, Cin, Cin, wx.data_ptr(), amx.data_ptr(), amw.data_ptr(),
                         bc.data_ptr(), y.data_ptr(), Cout, Cout, 0, None, 0, kc, amy.data_ptr(), _s())
    dx = torch.empty(N * H * H, Cin, device="cuda")
    L.cdm_conv3x3_fwd_h3(gyn.data_ptr(), N, H, H, Cout, Cout, wdx.data_ptr(), amg.data_ptr(), amd.data_ptr(), None,
                         dx.data_ptr(), Cin, Cin, 0, None, 0, kc, None, _s())
    torch.cuda.synchronize()
    assert amy.item() == y.abs().max().item()          # fused max|y| of the epilogue
    sp = L.raw("cdm_gemm_splits")(N * H * H, 5)
    slab = torch.empty(sp, Cout, 9 * Cin, device="cuda")
    L.cdm_conv3x3_wgrad_h3(gyn.data_ptr(), Cout, Cout, xn.data_ptr(), N, H, H, Cin, Cin, amg.data_ptr(),
                           amx.data_ptr(), sp, slab.data_ptr(), _s())
    dW = torch.empty(Cout, Cin, 3, 3, device="cuda")
    L.cdm_slab_reduce(slab.data_ptr(), sp, Cout, 9 * Cin, dW.data_ptr(), 9 * Cin, 1, 9, Cin, 0, 1.0, _s())
    torch.cuda.synchronize()
    return _nchw(y, N, H, H, Cout), _nchw(dx, N, H, H, Cin), dW


@pytest.mark.parametrize("N,H,Cin,Cout,kc", [(2, 16, 32, 64, 16), (1, 64, 128, 128, 16), (3, 8, 8, 16, 0),
                                              (2, 32, 256, 128, 16), (1, 8, 12, 20, 0), (1, 128, 128, 128, 16),
                                              (1, 256, 32, 128, 16), (2, 128, 64, 256, 16)])
def test_conv3x3_h3_fp32_class(L, N, H, Cin, Cout, kc):
    """h3 (scaled fp16 hi/lo, 3 products) fwd / dgrad / wgrad at the x6 (fp32) tolerance, and its relative-L2
    error vs an fp64 conv within 4x that of torch's own fp32 CPU conv on the same data.  (torch CPU sums in
    blocks; every MFMA path accumulates one fp32 chain per output.  Measured, profiles/r1_conv_accuracy.jsonl:
    x6 shows 1.1-3.9x torch's error, h3 0.4-3.0x — h3 is below x6 on every shape and pass.)"""
    torch.manual_seed(4)
    x = torch.randn(N, Cin, H, H).relu(); W = torch.randn(Cout, Cin, 3, 3) * 0.05; b = torch.randn(Cout)
    gy = torch.randn(N, Cout, H, H) * 1e-6          # gradient-like magnitudes (fp16 subnormal unscaled)
    y, dx, dW = _conv_h3(L, x, W, b, gy, kc)
    xd, Wd = x.double().requires_grad_(), W.double().requires_grad_()
    r64 = F.conv2d(xd, Wd, b.double(), padding=1)
    r64.backward(gy.double())
    xf, Wf = x.clone().requires_grad_(), W.clone().requires_grad_()
    r32 = F.conv2d(xf, Wf, b, padding=1)
    r32.backward(gy)
    for got, f32, f64 in ((y, r32.detach(), r64.detach()), (dx, xf.grad, xd.grad), (dW, Wf.grad, Wd.grad)):
        _close(got, f64.float(), 2e-5)
        e_h3 = (got.double().cpu() - f64).norm().item()
        e_32 = (f32.double() - f64).norm().item()
        assert e_h3 <= 4.0 * e_32 + 1e-12 * f64.norm().item(), (e_h3, e_32)


@pytest.mark.parametrize("xs,ws", [(1e-30, 1.0), (1e30, 1.0), (1.0, 1e-20), (1.0, 1e20), (1e-12, 1e9), (1.0, 1.0)])
def test_conv3x3_h3_scale_invariant(L, xs, ws):
    """The per-tensor power-of-two scaling keeps h3 fp32-class at any magnitude (fp16's own range is
    6e-5..65504), including a tensor whose channels span 1e-6..1e3 of its scale.  x ~ xs, W ~ ws, dY ~ 1/xs,
    so y, dx and dW all stay inside fp32's range."""
    torch.manual_seed(6)
    N, H, Cin, Cout = 2, 16, 32, 32
    x = torch.randn(N, Cin, H, H) * torch.logspace(-6, 3, Cin)[None, :, None, None] * xs
    W = torch.randn(Cout, Cin, 3, 3) * 0.05 * ws
    b = torch.zeros(Cout)
    gy = torch.randn(N, Cout, H, H) / xs
    y, dx, dW = _conv_h3(L, x, W, b, gy, 16)
    xd, Wd = x.double().requires_grad_(), W.double().requires_grad_()
    r = F.conv2d(xd, Wd, None, padding=1)
    r.backward(gy.double())
    for got, ref in ((y, r.detach()), (dx, xd.grad), (dW, Wd.grad)):
        got = got.double().cpu()
        assert torch.isfinite(got).all()
        err = (got - ref).abs().max().item() / ref.abs().max().item()
        assert err < 2e-5, err


def test_split_f16x2_terms(L):
    """hi + lo reproduces every weight to 2^-22 relative, or to half an fp16 subnormal step of the scaled
    tensor (2^-25 of the scale unit) for weights below 2^-17 max|w| (scaled by the power of two from max|w|)."""
    torch.manual_seed(5)
    K, NN = 40, 12
    w = (torch.randn(K, NN) * torch.logspace(-3, 3, K)[:, None]).cuda()
    xs, am = _split_h3(L, w, K, NN)
    assert am.item() == w.abs().max().item()
    t = xs.view(torch.float16).float().reshape(-1, 3, NN, 16)[:, :2]
    e = int(np.frexp(am.item())[1])
    rec = (t.double().sum(1).permute(0, 2, 1).reshape(-1, NN)[:K]) * 2.0 ** (e - 14)
    wd = w.double()
    bound = torch.maximum(2.0 ** -22 * wd.abs(), torch.full_like(wd, 2.0 ** (e - 14 - 25)))
    assert ((rec - wd).abs() <= bound).all()


@pytest.mark.parametrize("N,S,C,Cin", [(2, 64, 128, 128), (2, 32, 256, 128), (1, 32, 128, 256), (2, 32, 256, 256),
                                       (1, 128, 256, 128), (256, 64, 128, 128), (256, 32, 256, 256)])
def test_bn_bwd_fused_into_conv_staging_bit_exact(L, N, S, C, Cin):
    """Fused BN backward (dy computed while staging, never written) == norm_apply_bwd mode 0 then the h3
    convs, bit for bit: dgrad (LDS-halo kernel) and wgrad (kernel-row kernel) at the same operand scale; the
    scale comes from cdm_bn_bwd_amax_bound, which must bound max|dy|."""
    from cdm_amd.engine import wgrad_splits
    g_ = torch.Generator(device="cuda").manual_seed(5)
    P = N * S * S
    gr = torch.randn(P, C, device="cuda", generator=g_) * 1e-3
    y = torch.randn(P, C, device="cuda", generator=g_) * 2 + 0.3
    x = torch.randn(P, Cin, device="cuda", generator=g_).relu()
    co = [torch.randn(C, device="cuda", generator=g_) for _ in range(7)]
    co[3] = co[3].abs() + 0.1                                   # invstd > 0
    s_, t_, mean, invstd, A, B, Cc = co
    dy = torch.empty(P, C, device="cuda")
    am = torch.zeros(4, device="cuda")                          # [max|dy| exact, bound, max|g|, max|y|]
    L.cdm_norm_apply_bwd(0, gr.data_ptr(), C, y.data_ptr(), C, N, S, S, C, s_.data_ptr(), t_.data_ptr(), 0,
                         mean.data_ptr(), invstd.data_ptr(), 0, 1, None, 0, A.data_ptr(), B.data_ptr(), Cc.data_ptr(),
                         0, dy.data_ptr(), C, am.data_ptr(), _s())
    L.cdm_amax_f32(gr.data_ptr(), P, C, C, am.data_ptr() + 8, 0, _s())
    L.cdm_amax_f32(y.data_ptr(), P, C, C, am.data_ptr() + 12, 0, _s())
    L.cdm_bn_bwd_amax_bound(C, A.data_ptr(), B.data_ptr(), Cc.data_ptr(), mean.data_ptr(), invstd.data_ptr(),
                            am.data_ptr() + 8, am.data_ptr() + 12, am.data_ptr() + 4, _s())
    torch.cuda.synchronize()
    assert am[1].item() >= am[0].item() > 0
    dslot = am.data_ptr() + 4
    coefs = [t.data_ptr() for t in co]
    # dgrad: weights [Cin][C][3][3] as the dgrad of a conv C -> ... (dgrad maps C channels to Cin)
    W = torch.randn(C, Cin, 3, 3) * 0.05
    wdg = torch.empty(9 * C, Cin, device="cuda")
    L.cdm_pack_conv3x3(W.cuda().data_ptr(), torch.zeros(C, device="cuda").data_ptr(), Cin, C, None, None, None, None,
                       0.0, torch.empty(9 * Cin, C, device="cuda").data_ptr(), None, wdg.data_ptr(), 16, _s())
    wx, amw = _split_h3(L, wdg, 9 * C, Cin)
    ref = torch.empty(P, Cin, device="cuda"); got = torch.empty(P, Cin, device="cuda")
    a1 = torch.zeros(2, device="cuda")
    L.cdm_conv3x3_fwd_h3(dy.data_ptr(), N, S, S, C, C, wx.data_ptr(), dslot, amw.data_ptr(), None, ref.data_ptr(), Cin,
                         Cin, 0, None, 0, 16, a1.data_ptr(), _s())
    L.cdm_conv3x3_dgrad_h3_bnbwd(gr.data_ptr(), C, y.data_ptr(), C, *coefs, N, S, S, C, wx.data_ptr(), dslot,
                                 amw.data_ptr(), got.data_ptr(), Cin, Cin, 0, a1.data_ptr() + 4, _s())
    torch.cuda.synchronize()
    assert torch.equal(got, ref)
    assert a1[0].item() == a1[1].item() == ref.abs().max().item()
    # the same dgrad also storing the dy it stages (each element once, for the weight gradient): dy bit for bit
    dyo = torch.full((P, C), float("nan"), device="cuda"); got2 = torch.empty_like(got)
    L.cdm_conv3x3_dgrad_x16_bnbwd_dy(gr.data_ptr(), C, y.data_ptr(), C, *coefs, N, S, S, C, wx.data_ptr(), dslot,
                                     amw.data_ptr(), got2.data_ptr(), Cin, Cin, 0, None, dyo.data_ptr(), 4, 0, _s())
    torch.cuda.synchronize()
    assert torch.equal(got2, ref)
    assert torch.equal(dyo, dy)
    # wgrad of the conv Cin -> C that produced y: dW[co=C][tap*Cin+ci]
    amx = _amax(L, x, P, Cin)
    sp = wgrad_splits(P, C, 9 * Cin)
    s_ref = torch.empty(sp, C, 9 * Cin, device="cuda"); s_got = torch.full_like(s_ref, float("nan"))
    L.cdm_conv3x3_wgrad_h3(dy.data_ptr(), C, C, x.data_ptr(), N, S, S, Cin, Cin, dslot, amx.data_ptr(), sp,
                           s_ref.data_ptr(), _s())
    L.cdm_conv3x3_wgrad_h3_bnbwd(gr.data_ptr(), C, y.data_ptr(), C, *coefs, C, x.data_ptr(), N, S, S, Cin, Cin, dslot,
                                 amx.data_ptr(), sp, s_got.data_ptr(), _s())
    torch.cuda.synchronize()
    assert torch.equal(s_got, s_ref)


@pytest.mark.parametrize("N,H,Cin,pre", [(97, 64, 128, False), (66, 64, 128, True), (40, 32, 256, True),
                                         (2, 64, 128, False)])
def test_bf16_halo_conv_vs_fp64(L, N, H, Cin, pre):
    """The one-term (bf16, C4) LDS-halo forward — one barrier per chunk, halo prefetched two chunks ahead, several
    256-pixel tiles per block incl. a short last block (N=97: 1,552 tiles, 3 per block) — against an fp64 conv of the
    same bf16-rounded operands: only fp32 accumulation error may remain (<= 5e-6 max|ref|), with the BN-ReLU staging
    of the fused forward (pre: z = relu(y s + t) rounded to bf16) and the batch-statistics epilogue."""
    Cout = 128
    g_ = torch.Generator(device="cuda").manual_seed(13)
    P = N * H * H
    x = torch.randn(P, Cin, device="cuda", generator=g_)
    s_ = torch.rand(Cin, device="cuda", generator=g_) + 0.5
    t_ = torch.randn(Cin, device="cuda", generator=g_) * 0.3
    W = torch.randn(Cout, Cin, 3, 3, device="cuda", generator=g_) * 0.05
    b = torch.randn(Cout, device="cuda", generator=g_)
    wpk, _ = _pack3x3(L, W, b, 16)
    wx = _split(L, wpk, 9 * Cin, Cout)
    y = torch.full((P, Cout), float("nan"), device="cuda")
    stats = torch.zeros(P // 128, 2, Cout, device="cuda")
    assert L.cdm_conv3x3_fwd_x16_ex(x.data_ptr(), N, H, H, Cin, Cin, s_.data_ptr() if pre else None,
                                    t_.data_ptr() if pre else None, wx.data_ptr(), None, None, b.data_ptr(),
                                    y.data_ptr(), Cout, Cout, 0, stats.data_ptr(), Cout, 16, None, None, 0, 1, 0,
                                    _s()) == 0
    torch.cuda.synchronize()
    xin = x.double()
    if pre:
        xin = (xin * s_.double() + t_.double()).float().double().relu()
    xb = xin.float().bfloat16().double().cpu().reshape(N, H, H, Cin).permute(0, 3, 1, 2)
    Wb = W.bfloat16().double().cpu()
    ref = F.conv2d(xb, Wb, b.double().cpu(), padding=1).permute(0, 2, 3, 1).reshape(P, Cout)
    got = y.double().cpu()
    assert torch.isfinite(got).all()
    err = (got - ref).abs().max().item() / ref.abs().max().item()
    assert err <= 5e-6, err
    st = stats.double().cpu().sum(0)
    assert ((st[0] - ref.sum(0)).abs() <= 1e-5 * ref.abs().sum(0)).all()
    assert ((st[1] - (ref * ref).sum(0)).abs() <= 1e-5 * (ref * ref).sum(0)).all()


def test_deep_staging_bit_exact(L, tmp_path):
    """The two-deep staging schedule of the bf16 forward halo conv (the halo two chunks ahead, $CDM_HALO_DEEP) produces
    the one-ahead schedule's output bit for bit, the row forms of the C_in = 1 forward and C_out = 1 input gradient equal
    the flat-pixel kernels bit for bit ($CDM_ROW_KERNELS), and the fused weight gradients are reproducible across
    processes: two child processes (tests/_variant_worker.py), the library reading the switches once per process.
    Round 6: the second process also runs the previous schedules — the lock-step weight gradient ($CDM_WGRAD_STAGGER=0),
    the halo B fetched in the last kernel row ($CDM_HALO_BEARLY=0), the ConvT input gradient at three blocks per CU
    ($CDM_CONVT_DGRAD_MINB=3) — which must give the same bits (slabs, producer BN sums, outputs, statistics)."""
    import subprocess
    import sys
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_variant_worker.py")
    outs = []
    for deep in ("1", "0"):
        f = tmp_path / f"deep{deep}.pt"
        env = dict(os.environ, CDM_HALO_DEEP=deep, CDM_ROW_KERNELS=deep)
        if deep == "0":
            env.update(CDM_WGRAD_STAGGER="0", CDM_HALO_BEARLY="0", CDM_CONVT_DGRAD_MINB="3")
        r = subprocess.run([sys.executable, worker, str(f)], env=env, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        outs.append(torch.load(f))
    a, b = outs
    assert a.keys() == b.keys()
    for k in a:
        assert torch.isfinite(a[k]).all(), k
        assert torch.equal(a[k], b[k]), k


@pytest.mark.gpu
@pytest.mark.parametrize("N,tpb", [(2, 3), (3, 8), (1, 5)])
def test_halo_conv_tiles_per_block_bit_exact(L, N, tpb):
    """Blocks that loop over several 256-pixel tiles (next tile's first halo / B fetched during the last chunk)
    produce the one-tile-per-block result bit for bit, including a short last block (tiles % tpb != 0)."""
    H, C = 64, 128
    g_ = torch.Generator(device="cuda").manual_seed(11)
    P = N * H * H
    x = torch.randn(P, C, device="cuda", generator=g_).relu()
    W = torch.randn(9 * C, C, device="cuda", generator=g_) * 0.05
    wx, amw = _split_h3(L, W, 9 * C, C)
    amx = _amax(L, x, P, C)
    ref = torch.full((P, C), float("nan"), device="cuda"); got = torch.full_like(ref, float("nan"))
    for out, t in ((ref, 1), (got, tpb)):
        assert L.cdm_conv3x3_halo_ablate(1 | (t << 16), x.data_ptr(), N, H, C, C, wx.data_ptr(), amx.data_ptr(),
                                         amw.data_ptr(), out.data_ptr(), C, C, _s()) == 0
    torch.cuda.synchronize()
    assert torch.isfinite(ref).all()
    assert torch.equal(got, ref)


def test_conv3x3_h3_bench_launch_shape(L):
    """The C2 bench launch itself: N=256, 64x64, 128 -> 128 (4,096 256-pixel tiles, multi-tile blocks and the XCD
    remap of the LDS-halo kernel, split-K over 1 M pixels in the weight gradient) — fwd with the bias / BN-stats /
    max|y| epilogue, dgrad, wgrad against torch CPU (fp32 for fwd / dgrad at the 2e-5 bar; the weight gradient
    against an fp64 GEMM over all 1,048,576 pixels at 5e-5)."""
    from cdm_amd.engine import wgrad_splits
    N, H, C = 256, 64, 128
    P = N * H * H
    g = torch.Generator().manual_seed(13)
    x = torch.randn(N, C, H, H, generator=g).relu_()
    W = torch.randn(C, C, 3, 3, generator=g) * 0.05
    b = torch.randn(C, generator=g)
    gy = torch.randn(N, C, H, H, generator=g) * 1e-3
    Wc, bc = W.cuda(), b.cuda()
    wpk, wdg = _pack3x3(L, Wc, bc, 16)
    (wx, amw), (wdx, amd) = _split_h3(L, wpk, 9 * C, C), _split_h3(L, wdg, 9 * C, C)
    xn, gyn = _nhwc(x), _nhwc(gy)
    amx, amg = _amax(L, xn, P, C), _amax(L, gyn, P, C)
    y = torch.empty(P, C, device="cuda")
    stats = torch.zeros((P + 127) // 128, 2, C, device="cuda")
    amy = torch.zeros(1, device="cuda")
    L.cdm_conv3x3_fwd_h3(xn.data_ptr(), N, H, H, C, C, wx.data_ptr(), amx.data_ptr(), amw.data_ptr(), bc.data_ptr(),
                         y.data_ptr(), C, C, 0, stats.data_ptr(), C, 16, amy.data_ptr(), _s())
    dx = torch.empty(P, C, device="cuda")
    L.cdm_conv3x3_fwd_h3(gyn.data_ptr(), N, H, H, C, C, wdx.data_ptr(), amg.data_ptr(), amd.data_ptr(), None,
                         dx.data_ptr(), C, C, 0, None, 0, 16, None, _s())
    sp = wgrad_splits(P, C, 9 * C)
    slab = torch.full((sp, C, 9 * C), float("nan"), device="cuda")
    L.cdm_conv3x3_wgrad_h3(gyn.data_ptr(), C, C, xn.data_ptr(), N, H, H, C, C, amg.data_ptr(), amx.data_ptr(), sp,
                           slab.data_ptr(), _s())
    dW = torch.empty(C, C, 3, 3, device="cuda")
    L.cdm_slab_reduce(slab.data_ptr(), sp, C, 9 * C, dW.data_ptr(), 9 * C, 1, 9, C, 0, 1.0, _s())
    torch.cuda.synchronize()
    yc = y.cpu()
    assert amy.item() == yc.abs().max().item()
    with torch.no_grad():
        ref = F.conv2d(x, W, b, padding=1)                       # torch CPU fp32
        _close(yc.reshape(N, H, H, C).permute(0, 3, 1, 2), ref)
        yr = ref.permute(0, 2, 3, 1).reshape(P, C).double()
        st = stats.cpu().double().sum(0)
        _close(st[0], yr.sum(0), 1e-4)
        _close(st[1], (yr ** 2).sum(0), 1e-4)
        del ref, yr
        dref = torch.nn.grad.conv2d_input(x.shape, W, gy, padding=1)
        _close(_nchw(dx, N, H, H, C), dref)
        del dref
        # weight gradient in fp64: dW[co][ci][ky][kx] = sum_p gy[p][co] * x[p + (ky-1, kx-1)][ci]
        gyd = gy.permute(0, 2, 3, 1).reshape(P, C).double()
        xp = F.pad(x, (1, 1, 1, 1)).permute(0, 2, 3, 1).double()
        wref = torch.empty(C, C, 3, 3, dtype=torch.float64)
        for ky in range(3):
            for kx in range(3):
                xs = xp[:, ky:ky + H, kx:kx + H, :].reshape(P, C)
                wref[:, :, ky, kx] = gyd.t() @ xs
        _close(dW, wref.float(), 5e-5)


@pytest.mark.parametrize("nf", [8, 128])
def test_batched_repack_equals_per_layer(L, nf):
    """h3 train repack in 3 launches (cdm_pack_split_conv3x3_batch) == the per-layer pack + amax + split path, bit for
    bit: every split image (term planes 0 and 1; h3 leaves the x6 lo plane unused) and every max|W| (nf=8 covers the
    tap-major kc=0 K order, nf=128 the chunk-major one)."""
    import cdm_amd.engine as E
    from cdm_amd import ContextUnet
    torch.manual_seed(3)
    m = ContextUnet(1, nf, 6, 64, conv_math="h3").cuda()
    P = {k: v.detach() for k, v in list(m.named_parameters()) + list(m.named_buffers())}
    out = []
    for batched in (True, False):
        eng = E.UNetEngine(nf, 6, 64, "cuda", "h3")
        eng.batch_repack = batched
        eng.repack(P, True, _s())
        torch.cuda.synchronize()
        out.append({k: v.clone() for k, v in eng.pk.items() if k.endswith(("_x", "_amax"))})
    a, b = out
    shapes = {l.name: (l.cin, l.cout) for l in E.conv_layers(nf, 64) if l.cin > 1}
    shapes["out.0"] = (2 * nf, nf)
    n = 0
    for name, (cin, cout) in shapes.items():
        for kind, N in ((".wpk", cout), (".wdg", cin)):
            k = name + kind
            assert torch.equal(a[k + "_amax"], b[k + "_amax"]), k
            ta = a[k + "_x"].view(torch.int16).view(-1, 3, N * 16)[:, :2]
            tb = b[k + "_x"].view(torch.int16).view(-1, 3, N * 16)[:, :2]
            assert torch.equal(ta, tb), k
            n += 1
    assert n == 2 * len(shapes)


@pytest.mark.parametrize("B,C,k", [(1, 32, 16), (5, 48, 16), (16, 32, 32), (20, 16, 16)])
def test_up0_large_map_kernels(L, B, C, k):
    """cdm_up0_fwd / cdm_up0_wgrad (config-5 up0: ConvTranspose2d(C, C, k, k) on the 1x1 to_vec map, weights read in
    the reference layout) vs torch CPU conv_transpose2d in fp64; fp32 FMA summation -> the fp32 bar of this file.
    B = 20 > 16: the forward's second 16-sample pass (the weight gradient takes B <= 16 and raises above)."""
    torch.manual_seed(11)
    KK = k * k
    x = torch.randn(B, C, 1, 1, dtype=torch.float64)
    W = torch.randn(C, C, k, k, dtype=torch.float64) * 0.1
    b = torch.randn(C, dtype=torch.float64)
    gy = torch.randn(B, C, k, k, dtype=torch.float64)
    xg, Wg = x.clone().requires_grad_(), W.clone().requires_grad_()
    ref = F.conv_transpose2d(xg, Wg, b, stride=k)
    ref.backward(gy)
    xc = x.reshape(B, C).float().cuda()
    Wc, bc = W.float().cuda(), b.float().cuda()
    y = torch.full((B, KK, C), float("nan"), device="cuda")
    L.cdm_up0_fwd(xc.data_ptr(), B, C, Wc.data_ptr(), KK, bc.data_ptr(), y.data_ptr(), _s())
    torch.cuda.synchronize()
    _close(y.reshape(B, k, k, C).permute(0, 3, 1, 2), ref.detach())
    gyn = gy.permute(0, 2, 3, 1).reshape(B, KK, C).float().contiguous().cuda()     # NHWC [B][ij][co]
    dW = torch.full((C, C, k, k), float("nan"), device="cuda")
    if B > 16:
        with pytest.raises(Exception):
            L.cdm_up0_wgrad(xc.data_ptr(), B, C, gyn.data_ptr(), KK, dW.data_ptr(), _s())
        return
    L.cdm_up0_wgrad(xc.data_ptr(), B, C, gyn.data_ptr(), KK, dW.data_ptr(), _s())
    torch.cuda.synchronize()
    _close(dW, Wg.grad)


def test_cin1_wgrad_bn_backward_fused_bit_exact(L):
    """init_conv.conv1's weight gradient with its BatchNorm backward applied while reading g and y
    (cdm_conv3x3_cin1_wgrad_bnbwd) == the apply kernel (cdm_norm_apply_bwd mode 0) followed by
    cdm_conv3x3_cin1_wgrad, partial for partial (the same bn_bwd_elem expression, the same summation order)."""
    N, H, C = 3, 64, 128
    P = N * H * H
    g_ = torch.Generator(device="cuda").manual_seed(31)
    r = lambda *s: torch.randn(*s, device="cuda", generator=g_)   # noqa: E731
    gin, y, x = r(P, C), r(P, C), r(N, H, H)
    co = [r(C), r(C) * 0.1, r(C) * 0.2, r(C).abs() + 0.5, r(C), r(C) * 1e-3, r(C) * 1e-3]   # s t mean invstd A B Cc
    nch = (H * H + 127) // 128
    ref, got = (torch.full((N * nch * 10 * C,), float("nan"), device="cuda") for _ in range(2))
    dy = torch.empty(P, C, device="cuda")
    L.cdm_norm_apply_bwd(0, gin.data_ptr(), C, y.data_ptr(), C, N, H, H, C, co[0].data_ptr(), co[1].data_ptr(), 0,
                         co[2].data_ptr(), co[3].data_ptr(), 0, 1, None, 0, co[4].data_ptr(), co[5].data_ptr(),
                         co[6].data_ptr(), 0, dy.data_ptr(), C, None, _s())
    L.cdm_conv3x3_cin1_wgrad(dy.data_ptr(), C, x.data_ptr(), N, H, H, C, 128, ref.data_ptr(), _s())
    L.cdm_conv3x3_cin1_wgrad_bnbwd(gin.data_ptr(), C, y.data_ptr(), C, *[t.data_ptr() for t in co], x.data_ptr(), N, H,
                                   H, C, 128, got.data_ptr(), _s())
    torch.cuda.synchronize()
    assert torch.isfinite(ref).all() and torch.equal(got, ref)


@pytest.mark.parametrize("B,C,k", [(1, 64, 16), (5, 128, 32), (16, 64, 64)])
def test_up0_large_map_input_gradient(L, B, C, k):
    """cdm_up0_dgrad (config-5 up0 input gradient over W in place, dy transposed per sample to [B][C][KK]) + the slab
    fold vs torch CPU conv_transpose2d's input gradient in fp64, at the fp32 bar of this file."""
    torch.manual_seed(12)
    KK = k * k
    x = torch.randn(B, C, 1, 1, dtype=torch.float64, requires_grad=True)
    W = torch.randn(C, C, k, k, dtype=torch.float64) * 0.1
    gy = torch.randn(B, C, k, k, dtype=torch.float64)
    F.conv_transpose2d(x, W, None, stride=k).backward(gy)
    dyT = gy.reshape(B, C, KK).float().contiguous().cuda()            # [B][co][ij]
    Wc = W.float().cuda()
    sp = L.raw("cdm_up0_dgrad_splits")(C, KK)
    slab = torch.full((sp * B * C,), float("nan"), device="cuda")
    L.cdm_up0_dgrad(dyT.data_ptr(), B, C, Wc.data_ptr(), KK, slab.data_ptr(), _s())
    dx = torch.full((B, C), float("nan"), device="cuda")
    L.cdm_slab_reduce(slab.data_ptr(), sp, B, C, dx.data_ptr(), C, 0, 1, C, 0, 1.0, _s())
    torch.cuda.synchronize()
    _close(dx, x.grad.reshape(B, C))


@pytest.mark.parametrize("nterm", [4, 1])
@pytest.mark.parametrize("B,S,cin,cout", [(2, 64, 128, 128), (4, 64, 128, 128), (2, 32, 256, 256), (2, 32, 128, 256),
                                          (3, 32, 128, 128), (16, 64, 128, 128)])
def test_producer_bn_sums_in_wgrad(B, S, cin, cout, nterm):
    """cdm_conv3x3_wgrad_x16_ex with x_sums (PreBnReluSums): the producer's BatchNorm-backward sums accumulated while
    the weight gradient stages X = relu(y s + t) — S1 = sum g_pre, S2 = sum g_pre xhat, S5 = sum xhat per channel —
    vs the same sums in fp64 on the host, <= 1e-5 relative (fp32 partials per split, folded in fp64), for both 16-bit
    arithmetics and every K-step size (16, 32, 64 pixels per barrier: the shapes pick them); every block's partial row
    written (each X pixel is summed by exactly one of the 3 x gx blocks that stage it).
    The weight gradient itself must equal the call without sums bit for bit."""
    import cdm_amd
    from cdm_amd.engine import wgrad_splits
    L = cdm_amd.lib()
    st = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device="cuda").manual_seed(5)
    P = B * S * S
    y = torch.randn(P, cin, device="cuda", generator=g)
    gx = torch.randn(P, cin, device="cuda", generator=g)
    dy = torch.randn(P, cout, device="cuda", generator=g) * 1e-2
    s_ = torch.rand(cin, device="cuda", generator=g) + 0.5
    t_ = torch.randn(cin, device="cuda", generator=g) * 0.1
    mean = torch.randn(cin, device="cuda", generator=g) * 0.1
    inv = torch.rand(cin, device="cuda", generator=g) + 0.5
    am = torch.ones(4, device="cuda") * 8.0
    sp = wgrad_splits(P, cout, 9 * cin)
    nt = sp * 3 * (cout // 128)                     # one partial per block: split x kernel row x co tile
    slabs = []
    sums = torch.full((nt * 5 * cin,), float("nan"), device="cuda")
    for with_sums in (True, False):
        slab = torch.empty(sp * cout * 9 * cin, device="cuda")
        L.cdm_conv3x3_wgrad_x16_ex(dy.data_ptr(), cout, None, 0, None, None, None, None, None, None, None, cout,
                                   y.data_ptr(), B, S, S, cin, cin, s_.data_ptr(), t_.data_ptr(),
                                   gx.data_ptr() if with_sums else None, cin, mean.data_ptr() if with_sums else None,
                                   inv.data_ptr() if with_sums else None, sums.data_ptr() if with_sums else None,
                                   am.data_ptr(), am.data_ptr() + 4, sp, slab.data_ptr(), nterm, 0, st)
        slabs.append(slab)
    torch.cuda.synchronize()
    assert torch.equal(slabs[0], slabs[1])
    sm = sums.view(nt, 5, cin)
    assert not torch.isnan(sm).any()
    got = sm.double().sum(0)
    zp = y * s_ + t_
    gp = torch.where(zp > 0, gx, torch.zeros_like(gx)).double()
    xh = ((y - mean) * inv).double()
    ref = torch.stack([gp.sum(0), (gp * xh).sum(0), xh.sum(0)])
    g3 = torch.stack([got[0], got[1], got[4]])
    err = ((g3 - ref).abs().max(dim=1).values / ref.abs().max(dim=1).values).max().item()
    assert err <= 1e-5, err
    assert float(got[2].abs().max()) == 0 and float(got[3].abs().max()) == 0


@pytest.mark.parametrize("dt", [0, 3])
def test_bn_bwd_dy_pass_bit_exact(L, dt):
    """cdm_bn_bwd_dy (the C4 layers' separate BN-backward pass) == norm_apply_bwd mode 0 (the expression the fused
    staging uses) bit for bit: fp32 in / out, and bf16 g / y in, dy rounded to bf16 (round to nearest even)."""
    g_ = torch.Generator(device="cuda").manual_seed(7)
    N, S, C = 3, 32, 128
    P = N * S * S
    gr = torch.randn(P, C, device="cuda", generator=g_) * 1e-3
    y = torch.randn(P, C, device="cuda", generator=g_) * 2 + 0.3
    if dt & 1:
        gr, y = gr.bfloat16().float(), y.bfloat16().float()
    co = [torch.randn(C, device="cuda", generator=g_) for _ in range(7)]
    co[3] = co[3].abs() + 0.1
    s_, t_, mean, invstd, A, B, Cc = co
    ref = torch.empty(P, C, device="cuda")
    L.cdm_norm_apply_bwd(0, gr.data_ptr(), C, y.data_ptr(), C, N, S, S, C, s_.data_ptr(), t_.data_ptr(), 0,
                         mean.data_ptr(), invstd.data_ptr(), 0, 1, None, 0, A.data_ptr(), B.data_ptr(), Cc.data_ptr(),
                         0, ref.data_ptr(), C, None, _s())
    if dt & 1:
        gi, yi = gr.bfloat16(), y.bfloat16()
        out = torch.empty(P, C, device="cuda", dtype=torch.bfloat16)
    else:
        gi, yi = gr, y
        out = torch.empty(P, C, device="cuda")
    L.cdm_bn_bwd_dy(gi.data_ptr(), C, yi.data_ptr(), C, P, C, *[t.data_ptr() for t in co], out.data_ptr(), C, dt, _s())
    torch.cuda.synchronize()
    want = ref.bfloat16() if dt & 2 else ref
    assert torch.equal(out, want)


@pytest.mark.parametrize("N,H,C", [(2, 64, 128), (3, 32, 64), (2, 128, 32), (1, 16, 48)])
def test_conv_cout1_band(L, N, H, C):
    """out.3's C_out = 1 conv (the band kernel: a block stages 256 / W output rows' halo, C channels per slab through
    LDS) vs F.conv2d in fp32, plain and with out.1's GroupNorm + ReLU applied while staging; the 32-channel slab form
    ($CDM_COUT1_SLAB=32, C % 32 == 0) bit-identical to the default 16-channel form."""
    torch.manual_seed(5)
    z = torch.randn(N, C, H, H); w = torch.randn(1, C, 3, 3) * 0.1; b = torch.randn(1)
    gs = torch.rand(N, C) + 0.5; gt = torch.randn(N, C) * 0.1
    ref = F.conv2d(z, w, b, padding=1)
    ref_gn = F.conv2d(torch.relu(z * gs[:, :, None, None] + gt[:, :, None, None]), w, b, padding=1)
    zn = _nhwc(z)
    w9 = w.reshape(C, 9).contiguous().cuda(); bc = b.cuda(); gsc = gs.contiguous().cuda(); gtc = gt.contiguous().cuda()
    outs = {}
    for sl in ("32", "16"):
        os.environ["CDM_COUT1_SLAB"] = sl
        try:
            o = torch.empty(N, 1, H, H, device="cuda"); og = torch.empty_like(o)
            assert L.cdm_conv3x3_cout1_fwd(zn.data_ptr(), C, N, H, H, C, w9.data_ptr(), bc.data_ptr(), o.data_ptr(),
                                           _s()) == 0
            assert L.cdm_conv3x3_cout1_fwd_gn(zn.data_ptr(), C, N, H, H, C, gsc.data_ptr(), gtc.data_ptr(),
                                              w9.data_ptr(), bc.data_ptr(), og.data_ptr(), _s()) == 0
            torch.cuda.synchronize()
            outs[sl] = (o.cpu(), og.cpu())
        finally:
            del os.environ["CDM_COUT1_SLAB"]
    _close(outs["32"][0], ref)
    _close(outs["32"][1], ref_gn)
    assert torch.equal(outs["32"][0], outs["16"][0]) and torch.equal(outs["32"][1], outs["16"][1])
