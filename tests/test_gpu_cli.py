"""End-to-end CLI (train_diffusion.py LR EPOCHS T [NUM_PARAMS]) on synthetic maps, tiny config."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "camels-diffusion-model_amd", "train_diffusion.py")


@pytest.mark.parametrize("args,cond", [(["1e-3", "2", "20", "6"], True), (["1e-3", "2", "20"], False)])
def test_cli_trains_checkpoints_and_samples(tmp_path, args, cond):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    r = subprocess.run([sys.executable, CLI, *args, "--synthetic", "150", "--n-feat", "16", "--batch-size", "16",
                        "--n-samples", "3", "--out-root", str(tmp_path)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    dirs = os.listdir(tmp_path)
    assert len(dirs) == 1
    out = tmp_path / dirs[0]
    assert dirs[0].startswith("paper_lr_" if cond else "BIGnoiselr_")
    loss = np.load(out / "loss_log.npy")
    assert loss.shape == (2,) and np.isfinite(loss).all()
    ckpts = os.listdir(out / "weights")
    assert ckpts == (["model_epoch_2.pth"] if cond else [])
    rec = np.load(out / "reconstructed_images.npy")
    assert rec.shape == (3, 1, 64, 64) and np.isfinite(rec).all()
    pdf = np.load(out / "distribution_comparison.npz")          # train_diffusion.py:250 statistics
    assert pdf["train_pdf_mean"].shape == pdf["bin_mid"].shape
    pk = np.load(out / "power_spectrum_comparison.npz")
    assert pk["k"].shape == (47,) and np.isfinite(pk["gen_mean"]).all()
    if cond:
        sd = torch.load(out / "weights" / "model_epoch_2.pth", weights_only=True)
        assert len(sd) == 156
        assert np.load(out / "generated_samples.npy").shape == (3, 1, 64, 64)


def test_cli_reads_camels_files(tmp_path):
    """--data / --params: the reference's file formats (maps [N,256,256], params [N/15,6]) through the device
    preprocessing (cdm_amd.data), the param_min / param_max files and the seeded 90/10 split."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    g = np.random.default_rng(3)
    maps = (np.exp(g.normal(size=(30, 256, 256))) * 1e-4).astype(np.float32)
    params = g.uniform(0.1, 3.0, size=(2, 6))
    np.save(tmp_path / "maps.npy", maps)
    np.save(tmp_path / "params.npy", params)
    out_root = tmp_path / "out"
    r = subprocess.run([sys.executable, CLI, "1e-3", "1", "20", "6", "--data", str(tmp_path / "maps.npy"),
                        "--params", str(tmp_path / "params.npy"), "--n-feat", "16", "--batch-size", "8",
                        "--n-samples", "2", "--out-root", str(out_root)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    out = out_root / os.listdir(out_root)[0]
    np.testing.assert_array_equal(np.load(out / "param_min.npy"), params.min(0, keepdims=True))
    info = open(out / "dataset_info.txt").read()
    assert "Total dataset size: 30" in info and "Test dataset size: 3" in info
