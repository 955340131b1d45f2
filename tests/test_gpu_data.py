"""Device data pipeline (cdm_amd.data.preprocess_maps, csrc/data.hip) vs the reference's own lines
(code/train_diffusion_condition.py:137-144, executed by tests/golden/make_golden_data.py).

Tolerance: outputs lie in [0, 1]; the only arithmetic difference is log10f (HIP) vs numpy's float32 log10
(last-ulp) and the association of the 4-tap bilinear sum — max |d| <= 4e-6.  The global min / max and the
order of every other fp32 operation follow the reference.
"""
import os

import numpy as np
import pytest
import torch

from oracle import data_ref as D

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden", "data.npz")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("tag", ["shift", "pos"])
def test_preprocess_maps_matches_reference(tag):
    import cdm_amd.data as data
    fx = np.load(GOLD)
    got = data.preprocess_maps(fx[tag + "_raw"]).cpu().numpy()
    assert got.shape == fx[tag + "_out"].shape
    assert np.abs(got - fx[tag + "_out"]).max() <= 4e-6


@pytest.mark.parametrize("N,S,O", [(64, 256, 64), (5, 128, 64), (3, 64, 64), (2, 100, 64)])
def test_preprocess_maps_vs_oracle_shapes(N, S, O):
    """Other map sizes (incl. non-integer scale 100 -> 64, identity 64 -> 64) and many maps (chunking)."""
    import cdm_amd.data as data
    g = np.random.default_rng(N + S)
    raw = (np.exp(g.normal(size=(N, S, S))) * 1e-4 - 2e-5).astype(np.float32)
    got = data.preprocess_maps(raw, O, chunk=7).cpu().numpy()
    ref = D.preprocess_maps(raw, O).numpy()
    assert np.abs(got - ref).max() <= 4e-6
