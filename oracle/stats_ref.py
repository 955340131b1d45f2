"""CPU oracle (TEST INFRASTRUCTURE ONLY) for the sample-statistics row, SURVEY §8f #3: P(k) and PDF.

A numpy restatement of the reference's analysis functions, used by tests/ to check the HIP kernels of
``cdm_amd.stats`` (csrc/stats.hip).  Pinned to vectors produced by the reference itself
(tests/golden/make_golden_stats.py -> tests/golden/stats.npz, test_oracle_golden.py).  Nothing in the
shipped package imports this module.

  power_spectrum(box, dl)            code/diffusion_utilities.py:302-368  (ortho FFT, round(k/dk) bins)
  compare_power_spectra(o, g, dl)    code/diffusion_utilities.py:370-448  (mean / std over images)
  calculate_power_spectrum_2d(img)   code/sample_power_spectra.py:112-165 (unnormalised FFT, 20 log edges)
  compare_distributions(a, b)        code/train_diffusion.py:196-236      (per-image density histograms)
"""
from __future__ import annotations

import numpy as np


def power_spectrum(box, dl=1.0):
    """diffusion_utilities.py:302-368 (2-D and 3-D)."""
    box = np.asarray(box)
    dims = box.shape
    nd = len(dims)
    if nd not in (2, 3):
        raise ValueError("Input box must be 2D or 3D")
    ft = np.fft.fftn(box, norm="ortho")                                            # :322
    comps = [2 * np.pi * np.fft.fftfreq(d, dl) for d in dims]                       # :325-327
    grids = np.meshgrid(*comps, indexing="ij")                                      # :330-336
    kgrid = np.sqrt(sum(g ** 2 for g in grids))
    dk = 2 * np.pi / (np.min(dims) * dl)                                            # :339
    n_bins = int(np.ceil(np.max(kgrid) / dk)) + 1                                   # :340-341
    pk = np.zeros(n_bins)
    count = np.zeros(n_bins)
    kf = kgrid.flatten()
    pf = (np.abs(ft) ** 2).flatten()
    for i in range(len(kf)):                                                        # :352-356 (flat order)
        b = int(round(kf[i] / dk))
        if b < n_bins:
            pk[b] += pf[i]
            count[b] += 1
    ok = count > 0
    pk[ok] /= count[ok]                                                             # :359-360
    pk *= dl ** nd                                                                  # :363
    return np.arange(n_bins) * dk, pk                                               # :366


def compare_power_spectra(original_images, generated_images, dl=1.0):
    """diffusion_utilities.py:370-448 without the figure: (k, orig mean, gen mean, orig std, gen std)."""
    o = np.asarray(original_images)
    g = np.asarray(generated_images)
    if o.ndim == 4:
        o, g = o[:, 0], g[:, 0]                                                     # squeeze(1), :382-385
    n = min(len(o), len(g))
    ok_, op_, gk_, gp_ = [], [], [], []
    for i in range(n):
        k, p = power_spectrum(o[i], dl); ok_.append(k); op_.append(p)
        k, p = power_spectrum(g[i], dl); gk_.append(k); gp_.append(p)
    m = min(len(k) for k in ok_ + gk_)                                              # :408
    oa = np.array([p[:m] for p in op_]); ga = np.array([p[:m] for p in gp_])
    return ok_[0][:m], oa.mean(0), ga.mean(0), oa.std(0), ga.std(0)


def calculate_power_spectrum_2d(image, dl=1.0):
    """sample_power_spectra.py:112-165: k in cycles (fftfreq), bin edges in radians (as the reference)."""
    image = np.asarray(image)
    nx, ny = image.shape
    p2 = np.abs(np.fft.fftshift(np.fft.fft2(image))) ** 2                           # :128-132
    kx = np.fft.fftshift(np.fft.fftfreq(nx, dl)); ky = np.fft.fftshift(np.fft.fftfreq(ny, dl))
    kx2, ky2 = np.meshgrid(kx, ky, indexing="ij")
    k2 = np.sqrt(kx2 ** 2 + ky2 ** 2)                                               # :141-142
    kf, pf = k2.flatten(), p2.flatten()
    edges = np.logspace(np.log10(2 * np.pi / (nx * dl)), np.log10(np.pi / dl), 20)  # :149-151
    kc, pv = [], []
    for i in range(len(edges) - 1):                                                 # :157-163
        msk = (kf >= edges[i]) & (kf < edges[i + 1])
        if np.sum(msk) > 0:
            kc.append(np.mean(kf[msk])); pv.append(np.mean(pf[msk]))
    return np.array(kc), np.array(pv)


def pdf_edges(a, b, delta=0.01):
    """train_diffusion.py:197-200."""
    bmax = max(np.max(a), np.max(b))
    bmin = min(np.min(a), np.min(b))
    return np.arange(bmin, bmax + delta, delta)


def compare_distributions(camels_images, diffusion_images):
    """train_diffusion.py:196-215 without the figure: (bin_mid, train mean, train std, test mean, test std)."""
    a, b = np.asarray(camels_images), np.asarray(diffusion_images)
    bins = pdf_edges(a, b)
    tr = np.array([np.histogram(a[i].ravel(), bins, density=True)[0] for i in range(len(a))])
    te = np.array([np.histogram(b[i].ravel(), bins, density=True)[0] for i in range(len(a))])
    mid = (bins[:-1] + bins[1:]) / 2.0
    return mid, tr.mean(0), tr.std(0), te.mean(0), te.std(0)
