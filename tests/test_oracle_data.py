"""Data-pipeline row on the CPU: the oracle and the host-side helpers of cdm_amd.data against
vectors produced by executing the reference's own lines (tests/golden/make_golden_data.py) — bit-exact."""
import os

import numpy as np
import pytest

from oracle import data_ref as D

GOLD = os.path.join(os.path.dirname(__file__), "golden", "data.npz")


@pytest.fixture(scope="module")
def fx():
    return np.load(GOLD)


@pytest.mark.parametrize("tag", ["shift", "pos"])
def test_oracle_preprocess_maps_bit_exact(fx, tag):
    np.testing.assert_array_equal(D.preprocess_maps(fx[tag + "_raw"]).numpy(), fx[tag + "_out"])


@pytest.mark.parametrize("num_params", [6, 4])
def test_preprocess_params_bit_exact(fx, num_params, tmp_path):
    import cdm_amd.data as data
    got = data.preprocess_params(fx["params_raw"], 30, num_params, str(tmp_path)).numpy()
    np.testing.assert_array_equal(got, fx[f"params_norm_{num_params}"].astype(np.float32))
    np.testing.assert_array_equal(np.load(tmp_path / "param_min.npy"), fx["param_min"])
    np.testing.assert_array_equal(np.load(tmp_path / "param_max.npy"), fx["param_max"])


def test_train_test_split_matches_random_split(fx):
    import cdm_amd.data as data
    tr, te = data.train_test_split(int(fx["split_n"]), 1500, 42)
    np.testing.assert_array_equal(tr.numpy(), fx["split_train"])
    np.testing.assert_array_equal(te.numpy(), fx["split_test"])


def test_params_txt_to_npy_roundtrip(tmp_path):
    """code/txt-npy.py: the same float64 table as np.loadtxt, written as .npy (CPU host helper)."""
    import cdm_amd.data as data
    tab = np.random.default_rng(0).uniform(0.1, 3.0, size=(10, 6))
    np.savetxt(tmp_path / "param.txt", tab)
    got = data.params_txt_to_npy(str(tmp_path / "param.txt"), str(tmp_path / "params.npy"))
    np.testing.assert_array_equal(got, np.loadtxt(tmp_path / "param.txt"))
    np.testing.assert_array_equal(np.load(tmp_path / "params.npy"), got)
    assert got.shape == (10, 6) and got.dtype == np.float64
