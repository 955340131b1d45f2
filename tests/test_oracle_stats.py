"""The CPU oracle of the sample-statistics row (oracle/stats_ref.py) against vectors produced by the
reference itself (tests/golden/make_golden_stats.py): P(k) and PDF, fp64 numpy, tolerance 1e-12 relative."""
import os

import numpy as np
import pytest

from oracle import stats_ref as S

GOLD = os.path.join(os.path.dirname(__file__), "golden", "stats.npz")


@pytest.fixture(scope="module")
def fx():
    return np.load(GOLD)


def _close(a, b, tol=1e-12):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    assert a.shape == b.shape, (a.shape, b.shape)
    assert np.abs(a - b).max() <= tol * max(np.abs(b).max(), 1e-300)


@pytest.mark.parametrize("tag,box", [("ps_a", "orig0"), ("ps_b", "gen1"), ("ps_c", "box32")])
def test_power_spectrum(fx, tag, box):
    img = {"orig0": fx["orig"][0], "gen1": fx["gen"][1], "box32": fx["box32"]}[box]
    k, pk = S.power_spectrum(img, float(fx[tag + "_dl"]))
    _close(k, fx[tag + "_k"])
    _close(pk, fx[tag + "_pk"])


def test_compare_power_spectra(fx):
    k, om, gm, os_, gs = S.compare_power_spectra(fx["orig"][:, None], fx["gen"][:, None], 1.0)
    _close(k, fx["cps_k"])
    _close(om, fx["cps_orig_mean"])
    _close(gm, fx["cps_gen_mean"])
    _close(os_[1:], fx["cps_orig_std"], 1e-10)      # recovered from the reference's (mean +- std) band
    _close(gs[1:], fx["cps_gen_std"], 1e-10)


@pytest.mark.parametrize("tag,img", [("p2d_a", ("orig", 2)), ("p2d_b", ("gen", 3))])
def test_calculate_power_spectrum_2d(fx, tag, img):
    k, pk = S.calculate_power_spectrum_2d(fx[img[0]][img[1]], float(fx[tag + "_dl"]))
    _close(k, fx[tag + "_k"])
    _close(pk, fx[tag + "_pk"])


def test_compare_distributions(fx):
    mid, trm, trs, tem, tes = S.compare_distributions(fx["orig"], fx["gen"])
    _close(mid, fx["pdf_bin_mid"])
    _close(trm, fx["pdf_train_mean"])
    _close(trs, fx["pdf_train_std"])
    _close(tem, fx["pdf_test_mean"])
    _close(tes, fx["pdf_test_std"])


@pytest.mark.parametrize("tag", ["ps3_a", "ps3_b", "ps_ns"])
def test_power_spectrum_3d_and_non_square(fx, tag):
    """The 3-D branch and a non-square 2-D box of power_spectrum (diffusion_utilities.py:316-363)."""
    k, pk = S.power_spectrum(fx[tag + "_box"], float(fx[tag + "_dl"]))
    _close(k, fx[tag + "_k"])
    _close(pk, fx[tag + "_pk"])
