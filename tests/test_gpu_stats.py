"""Sample-statistics row on the HIP kernels vs the reference's golden vectors and the CPU oracle.

The HIP path computes in fp64 (direct DFT).  The reference's numpy 2.x FFT keeps the precision of its input,
so on float32 maps the reference itself works in complex64.  Hence two bars, per element:
  vs an fp64 evaluation of the reference formula (oracle on float64 input)  |d| <= 1e-12 max|ref| + 1e-9 |ref|
  vs the reference's own golden values (complex64 FFT)                      |d| <= 1e-7 max|ref| + 2e-5 |ref|
  bin geometry (k axes, bin membership / counts): exact.  PDFs: fp64 both sides, 1e-12 / 1e-9.
"""
import os

import numpy as np
import pytest
import torch

from oracle import stats_ref as S

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden", "stats.npz")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.fixture(scope="module")
def fx():
    return np.load(GOLD)


F32REF = dict(rel=2e-5, absmax=1e-7)        # vs the reference's complex64 FFT


def _close(a, b, rel=1e-9, absmax=1e-12):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    assert a.shape == b.shape, (a.shape, b.shape)
    bound = absmax * max(np.abs(b).max(), 1e-300) + rel * np.abs(b)
    bad = np.abs(a - b) > bound
    assert not bad.any(), (np.abs(a - b)[bad][:5], b[bad][:5])


@pytest.mark.parametrize("tag,box", [("ps_a", "orig0"), ("ps_b", "gen1"), ("ps_c", "box32")])
def test_power_spectrum_matches_reference(fx, tag, box):
    import cdm_amd
    img = {"orig0": fx["orig"][0], "gen1": fx["gen"][1], "box32": fx["box32"]}[box]
    dl = float(fx[tag + "_dl"])
    k, pk = cdm_amd.power_spectrum(img, dl)
    np.testing.assert_array_equal(k, fx[tag + "_k"])
    _close(pk, fx[tag + "_pk"], **F32REF)
    _close(pk, S.power_spectrum(img.astype(np.float64), dl)[1])


@pytest.mark.parametrize("tag", ["ps3_a", "ps3_b", "ps_ns"])
def test_power_spectrum_3d_and_non_square(fx, tag):
    """3-D boxes (16x20x24 at dl=0.5, 24^3) and a 24x40 map: the per-axis DFT path (cdm_dftn_power) vs the
    reference's own values and the fp64 oracle."""
    import cdm_amd
    box, dl = fx[tag + "_box"], float(fx[tag + "_dl"])
    k, pk = cdm_amd.power_spectrum(box, dl)
    np.testing.assert_array_equal(k, fx[tag + "_k"])
    _close(pk, fx[tag + "_pk"], **F32REF)
    _close(pk, S.power_spectrum(box.astype(np.float64), dl)[1])


def test_compare_power_spectra_matches_reference(fx, tmp_path):
    import cdm_amd
    k, om, gm = cdm_amd.compare_power_spectra(torch.from_numpy(fx["orig"][:, None]),
                                              torch.from_numpy(fx["gen"][:, None]), str(tmp_path), dl=1.0)
    np.testing.assert_array_equal(k, fx["cps_k"])
    _close(om, fx["cps_orig_mean"], **F32REF)
    _close(gm, fx["cps_gen_mean"], **F32REF)
    saved = np.load(tmp_path / "power_spectrum_comparison.npz")
    _close(saved["orig_std"][1:], fx["cps_orig_std"], rel=1e-4, absmax=1e-6)
    _close(saved["gen_std"][1:], fx["cps_gen_std"], rel=1e-4, absmax=1e-6)
    _, om64, gm64, os64, gs64 = S.compare_power_spectra(fx["orig"].astype(np.float64), fx["gen"].astype(np.float64))
    _close(om, om64); _close(gm, gm64)
    _close(saved["orig_std"], os64, rel=1e-8); _close(saved["gen_std"], gs64, rel=1e-8)


@pytest.mark.parametrize("tag,img", [("p2d_a", ("orig", 2)), ("p2d_b", ("gen", 3))])
def test_calculate_power_spectrum_2d_matches_reference(fx, tag, img):
    import cdm_amd
    im, dl = fx[img[0]][img[1]], float(fx[tag + "_dl"])
    k, pk = cdm_amd.calculate_power_spectrum_2d(im, dl)
    _close(k, fx[tag + "_k"], rel=1e-15)
    _close(pk, fx[tag + "_pk"], **F32REF)
    _close(pk, S.calculate_power_spectrum_2d(im.astype(np.float64), dl)[1])


def test_compare_distributions_matches_reference(fx, tmp_path):
    import cdm_amd
    r = cdm_amd.compare_distributions(fx["orig"], fx["gen"], str(tmp_path))
    _close(r["bin_mid"], fx["pdf_bin_mid"], rel=0, absmax=0)
    for k, g in (("train_pdf_mean", "pdf_train_mean"), ("train_pdf_std", "pdf_train_std"),
                 ("test_pdf_mean", "pdf_test_mean"), ("test_pdf_std", "pdf_test_std")):
        _close(r[k], fx[g])
    assert (tmp_path / "distribution_comparison.npz").exists()


@pytest.mark.parametrize("N,B", [(64, 256), (256, 4), (48, 3)])
def test_power_spectra_batched_vs_oracle(N, B):
    """Full-size batches (bench shapes: 256 maps of 64x64; C5 maps 256x256) against the numpy oracle."""
    import cdm_amd
    g = torch.Generator().manual_seed(N + B)
    x = torch.rand(B, 1, N, N, generator=g)
    k, pk = cdm_amd.power_spectra(x.cuda(), dl=0.75)
    pk = pk.cpu().numpy()
    for b in ([0, B - 1] if B > 2 else range(B)):
        kr, pr = S.power_spectrum(x[b, 0].numpy().astype(np.float64), 0.75)
        np.testing.assert_array_equal(k, kr)
        _close(pk[b], pr)


def test_pdfs_edges_and_ranges_vs_numpy():
    """np.histogram(density=True) semantics: closed last bin, out-of-range values dropped, edge hits."""
    import cdm_amd
    g = torch.Generator().manual_seed(3)
    x = torch.rand(5, 64, 64, generator=g) * 1.2 - 0.1
    x[0, 0, :8] = torch.tensor([0.0, 0.5, 1.0, -0.1, 1.1, 0.25, 0.75, 0.3])
    edges = np.arange(0.0, 1.0 + 0.01, 0.01)
    got = cdm_amd.pdfs(x, edges).cpu().numpy()
    for b in range(5):
        ref = np.histogram(x[b].numpy().ravel(), edges, density=True)[0]
        _close(got[b], ref)


@pytest.mark.parametrize("shape", [(32, 32), (16, 20, 24), (24, 40)])
def test_power_spectrum_fp64_box(shape):
    """a float64 box (values not representable in fp32) keeps fp64 input, as np.fft.fftn computes on it
    (diffusion_utilities.py:322): HIP vs the fp64 oracle at the fp64 bar; a CUDA tensor input is used on its device."""
    import cdm_amd
    box = np.random.default_rng(7).standard_normal(shape) * (1 + 1e-9)
    assert not np.array_equal(box.astype(np.float32).astype(np.float64), box)
    k, pk = cdm_amd.power_spectrum(box, 0.5)
    kr, pr = S.power_spectrum(box, 0.5)
    np.testing.assert_array_equal(k, kr)
    _close(pk, pr)
    k2, pk2 = cdm_amd.power_spectrum(torch.from_numpy(box).cuda(), 0.5)
    np.testing.assert_array_equal(pk2, pk)
