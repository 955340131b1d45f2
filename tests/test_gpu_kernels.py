"""Op-level parity of the HIP contraction kernels against plain torch fp32 on CPU (GPU box only).

Tolerance: fp32 MFMA vs CPU fp32 with different summation order -> |err| <= 2e-5 * max|ref| + 1e-5.
"""
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


@pytest.mark.parametrize("N,Hin,Cin,Cout", [(2, 8, 64, 32), (1, 16, 512, 128), (3, 4, 16, 8)])
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
    L.cdm_convT2x2_fwd(xn.data_ptr(), N, Hin, Hin, Cin, Cin, wt.data_ptr(), bc.data_ptr(), y.data_ptr(), Cout, Cout,
                       _s())
    torch.cuda.synchronize()
    _close(_nchw(y, N, 2 * Hin, 2 * Hin, Cout), ref.detach())
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
