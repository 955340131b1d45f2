"""Sample statistics of maps on the HIP kernels: power spectrum P(k) and PDFs.

Reference functions (same names, arguments and return values; the matplotlib figures are replaced by an
optional ``.npz`` of the plotted arrays in ``output_dir``):
  power_spectrum(box, dl=1.0) -> (k_bins, pk)               code/diffusion_utilities.py:302-368
  compare_power_spectra(original_images, generated_images, output_dir, dl=1.0, title=...)
      -> (k, orig_pk_mean, gen_pk_mean)                      code/diffusion_utilities.py:370-448
  calculate_power_spectrum_2d(image, dl=1.0) -> (k, pk)     code/sample_power_spectra.py:112-165
  compare_distributions(camels_images, diffusion_images, output_dir)   code/train_diffusion.py:196-236
      -> dict(bin_mid, train_pdf_mean, train_pdf_std, test_pdf_mean, test_pdf_std)
Batched device entry points: ``power_spectra(images, dl)`` ([B, N, N] -> [B, nbins] fp64) and
``pdfs(images, edges)`` ([B, ...] -> [B, nbins] fp64 densities).

Split of work: the per-map O(N^3) fp64 DFT + |F|^2, the per-bin power sums and the per-map histograms run
in csrc/stats.hip; the bin geometry (which frequency goes to which bin, in the reference's summation
order) depends only on N and dl and is built once on the host with the reference's own expressions.
power_spectrum also takes 3-D and non-square 2-D boxes (its reference branch at diffusion_utilities.py:316-336): one
direct-DFT pass per axis (cdm_dftn_power) and the same host-built bin geometry.
"""
from __future__ import annotations

import os
from functools import lru_cache
from typing import Tuple

import numpy as np
import torch

from ._lib import lib


def _s():
    return torch.cuda.current_stream().cuda_stream


@lru_cache(maxsize=16)
def _radial_geometry(dims, dl: float):
    """power_spectrum's bins (diffusion_utilities.py:325-341) for a box of extents ``dims`` (2-D or 3-D): CSR lists of
    flat indices per bin, flat order."""
    if isinstance(dims, int):
        dims = (dims, dims)
    comps = [2 * np.pi * np.fft.fftfreq(d, dl) for d in dims]
    grids = np.meshgrid(*comps, indexing="ij")
    kgrid = np.sqrt(sum(g ** 2 for g in grids))      # kx**2 + ky**2 (+ kz**2), the reference's order of additions
    dk = 2 * np.pi / (np.min(dims) * dl)
    n_bins = int(np.ceil(np.max(kgrid) / dk)) + 1
    kf = kgrid.flatten()
    bins = np.array([int(round(v / dk)) for v in kf])
    keep = bins < n_bins
    order = np.arange(kf.size)[keep]
    b = bins[keep]
    srt = np.argsort(b, kind="stable")                 # stable: flat order inside each bin
    idx = order[srt].astype(np.int32)
    off = np.zeros(n_bins + 1, np.int32)
    np.add.at(off, b + 1, 1)
    off = np.cumsum(off).astype(np.int32)
    count = np.diff(off).astype(np.float64)
    return np.arange(n_bins) * dk, idx, off, count


@lru_cache(maxsize=16)
def _log_geometry(N: int, dl: float):
    """calculate_power_spectrum_2d's bins (sample_power_spectra.py:134-163), indices into the unshifted
    spectrum listed in the order of the reference's fftshifted flat arrays."""
    kx = np.fft.fftshift(np.fft.fftfreq(N, dl))
    kx2, ky2 = np.meshgrid(kx, kx, indexing="ij")
    kf = np.sqrt(kx2 ** 2 + ky2 ** 2).flatten()
    sh = np.fft.fftshift(np.arange(N * N).reshape(N, N)).flatten()   # shifted flat pos -> unshifted index
    edges = np.logspace(np.log10(2 * np.pi / (N * dl)), np.log10(np.pi / dl), 20)
    lists, kc = [], []
    for i in range(len(edges) - 1):
        m = (kf >= edges[i]) & (kf < edges[i + 1])
        if np.sum(m) > 0:
            lists.append(sh[m]); kc.append(np.mean(kf[m]))
    off = np.zeros(len(lists) + 1, np.int32)
    off[1:] = np.cumsum([len(x) for x in lists])
    idx = np.concatenate(lists).astype(np.int32) if lists else np.zeros(0, np.int32)
    return np.array(kc), idx, off, np.diff(off).astype(np.float64)


def _as_maps(images) -> torch.Tensor:
    x = torch.as_tensor(images)
    if x.dim() == 4:
        x = x[:, 0]                                          # [B, 1, H, W] -> [B, H, W] (squeeze(1))
    if x.dim() == 2:
        x = x[None]
    if x.dim() != 3 or x.shape[1] != x.shape[2]:
        raise ValueError("expected square 2-D maps [B, N, N] / [B, 1, N, N] / [N, N]")
    return x.to(x.device if x.is_cuda else "cuda", torch.float32).contiguous()


def _power(x: torch.Tensor, scale: float) -> torch.Tensor:
    B, N = x.shape[0], x.shape[1]
    T = torch.empty(B * N * N * 2, dtype=torch.float64, device=x.device)
    P = torch.empty(B, N, N, dtype=torch.float64, device=x.device)
    lib().cdm_dft2_power(x.data_ptr(), B, N, float(scale), T.data_ptr(), P.data_ptr(), _s())
    return P


def _bin_sums(P: torch.Tensor, idx: np.ndarray, off: np.ndarray) -> torch.Tensor:
    B, NN = P.shape[0], P[0].numel()
    nb = len(off) - 1
    di = torch.from_numpy(idx).to(P.device)
    do = torch.from_numpy(off).to(P.device)
    out = torch.empty(B, nb, dtype=torch.float64, device=P.device)
    lib().cdm_bin_sum(P.data_ptr(), B, NN, do.data_ptr(), di.data_ptr(), nb, out.data_ptr(), _s())
    torch.cuda.current_stream().synchronize()               # di / do are temporaries
    return out


def _power_nd(x: torch.Tensor, dims, scale: float) -> torch.Tensor:
    """|fftn|^2 * scale of B boxes x [B, *dims] (any rank <= 3, any extents; fp32 or fp64): one DFT pass per axis."""
    import ctypes
    B = x.shape[0]
    n = int(np.prod(dims))
    T0 = torch.empty(B * n * 2, dtype=torch.float64, device=x.device)
    T1 = torch.empty(B * n * 2, dtype=torch.float64, device=x.device) if len(dims) > 2 else T0
    P = torch.empty(B, n, dtype=torch.float64, device=x.device)
    d = (ctypes.c_int * len(dims))(*dims)          # read by the host entry point before it returns
    fn = lib().cdm_dftn_power_f64 if x.dtype == torch.float64 else lib().cdm_dftn_power
    fn(x.data_ptr(), B, len(dims), ctypes.addressof(d), float(scale), T0.data_ptr(), T1.data_ptr(), P.data_ptr(), _s())
    return P


def _binned(P: torch.Tensor, dims, dl: float):
    k, idx, off, count = _radial_geometry(tuple(dims), float(dl))
    s = _bin_sums(P, idx, off)
    cnt = torch.from_numpy(count).to(s.device)
    return k, torch.where(cnt > 0, s / cnt.clamp(min=1), s) * (dl ** len(dims))   # :359-363


def power_spectra(images, dl: float = 1.0) -> Tuple[np.ndarray, torch.Tensor]:
    """Batched power_spectrum of square 2-D maps: (k_bins [nbins], pk [B, nbins] fp64 on the device)."""
    x = _as_maps(images)
    N = x.shape[1]
    P = _power(x, 1.0 / (N * N))                            # |fftn(norm="ortho")|^2 = |F|^2 / N^2
    return _binned(P, (N, N), dl)


def power_spectrum(box, dl: float = 1.0):
    """diffusion_utilities.py:302-368 for a 2-D or 3-D box (any extents) -> (k_bins, pk) numpy."""
    x = box if torch.is_tensor(box) else torch.from_numpy(np.asarray(box))
    if x.dim() not in (2, 3):
        raise ValueError("Input box must be 2D or 3D")
    # np.fft.fftn computes in the input's precision: fp64 boxes (numpy's default) keep fp64 values, anything else fp32;
    # a CUDA tensor stays on its device
    f64 = x.dtype == torch.float64
    if x.dim() == 2 and x.shape[0] == x.shape[1] and not f64:
        k, pk = power_spectra(x, dl)
        return k, pk[0].cpu().numpy()
    dims = tuple(int(v) for v in x.shape)
    dev = x.device if x.is_cuda else torch.device("cuda")
    x = x.detach().to(dev, torch.float64 if f64 else torch.float32).contiguous().reshape(1, -1)
    P = _power_nd(x, dims, 1.0 / float(np.prod(dims)))      # norm="ortho": |F|^2 / prod(dims)
    k, pk = _binned(P, dims, dl)
    return k, pk[0].cpu().numpy()


def compare_power_spectra(original_images, generated_images, output_dir=None, dl: float = 1.0,
                          title: str = "Power Spectrum Comparison"):
    """diffusion_utilities.py:370-448 -> (k, orig_pk_mean, gen_pk_mean); arrays (incl. std) -> .npz."""
    o, g = _as_maps(original_images), _as_maps(generated_images)
    n = min(o.shape[0], g.shape[0])
    k, po = power_spectra(o[:n], dl)
    _, pg = power_spectra(g[:n], dl)
    po, pg = po.cpu().numpy(), pg.cpu().numpy()
    om, gm, osd, gsd = po.mean(0), pg.mean(0), po.std(0), pg.std(0)
    if output_dir is not None:
        os.makedirs(output_dir, exist_ok=True)
        np.savez(os.path.join(output_dir, "power_spectrum_comparison.npz"), k=k, orig_mean=om, orig_std=osd,
                 gen_mean=gm, gen_std=gsd, title=title)
    return k, om, gm


def calculate_power_spectrum_2d(image, dl: float = 1.0):
    """sample_power_spectra.py:112-165 -> (k_centers, pk) numpy (unnormalised FFT, 20 log-spaced edges)."""
    x = _as_maps(image)
    if x.shape[0] != 1:
        raise ValueError("one 2-D image")
    N = x.shape[1]
    kc, idx, off, count = _log_geometry(N, float(dl))
    if len(kc) == 0:
        return kc, np.zeros(0)
    s = _bin_sums(_power(x, 1.0), idx, off)
    return kc, s[0].cpu().numpy() / count


def pdfs(images, edges) -> torch.Tensor:
    """Per-map np.histogram(map.ravel(), edges, density=True) -> [B, len(edges) - 1] fp64 on the device."""
    x = torch.as_tensor(images)
    B = x.shape[0]
    x = x.reshape(B, -1).to("cuda", torch.float32).contiguous()
    e = torch.as_tensor(np.asarray(edges, np.float64)).to(x.device)
    nb = e.numel() - 1
    out = torch.empty(B, nb, dtype=torch.float64, device=x.device)
    lib().cdm_histogram_density(x.data_ptr(), B, x.shape[1], e.data_ptr(), nb, out.data_ptr(), _s())
    torch.cuda.current_stream().synchronize()
    return out


def compare_distributions(camels_images, diffusion_images, output_dir=None):
    """train_diffusion.py:196-236: per-map PDFs on 0.01 bins spanning both sets; mean / std over maps."""
    a = camels_images.detach().cpu().numpy() if torch.is_tensor(camels_images) else np.asarray(camels_images)
    b = diffusion_images.detach().cpu().numpy() if torch.is_tensor(diffusion_images) else np.asarray(diffusion_images)
    bin_max = max(a.max(), b.max())
    bin_min = min(a.min(), b.min())
    bins = np.arange(bin_min, bin_max + 0.01, 0.01)                                   # :197-200
    n = len(a)
    tr = pdfs(a[:n], bins).cpu().numpy()
    te = pdfs(b[:n], bins).cpu().numpy()
    res = {"bin_mid": (bins[:-1] + bins[1:]) / 2.0, "train_pdf_mean": tr.mean(0), "train_pdf_std": tr.std(0),
           "test_pdf_mean": te.mean(0), "test_pdf_std": te.std(0)}
    if output_dir is not None:
        os.makedirs(output_dir, exist_ok=True)
        np.savez(os.path.join(output_dir, "distribution_comparison.npz"), **res)
    return res
