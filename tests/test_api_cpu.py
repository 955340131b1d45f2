"""Drop-in API surface on CPU: constructor signatures, attributes, state_dict layout, seeded init,
reference-named shims, C-ABI library exports every header symbol (no GPU compute here)."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_contextunet_signature_and_attributes():
    import cdm_amd
    m = cdm_amd.ContextUnet(1, n_feat=16, n_cfeat=6, height=64)
    assert (m.in_channels, m.n_feat, m.n_cfeat, m.h) == (1, 16, 6, 64)
    m2 = cdm_amd.ContextUnet(1)
    assert (m2.n_feat, m2.n_cfeat, m2.h) == (128, 10, 64)          # reference defaults (ContextUnet.py:6)
    sd = m.state_dict()
    assert len(sd) == 156 and sd["init_conv.conv1.1.num_batches_tracked"].dtype == torch.int64


def test_seeded_init_equals_reference(golden_dir):
    import cdm_amd
    fx = np.load(os.path.join(golden_dir, "model_nf16.npz"))
    torch.manual_seed(0)
    m = cdm_amd.ContextUnet(1, 16, 6, 64)
    for k, v in m.state_dict().items():
        assert np.array_equal(v.numpy(), fx["sd." + k]), k


def test_block_constructors():
    import cdm_amd
    b = cdm_amd.ResidualConvBlock(3, 8, is_res=True)
    assert b.is_res and not b.same_channels and b.get_out_channels() == 8
    assert isinstance(cdm_amd.UnetUp(16, 8).model[0], torch.nn.ConvTranspose2d)
    assert isinstance(cdm_amd.UnetDown(8, 16).model[2], torch.nn.MaxPool2d)
    assert cdm_amd.EmbedFC(6, 32).input_dim == 6


def test_reference_named_shims():
    code = ("import sys; sys.path.insert(0, %r); from ContextUnet import ContextUnet; "
            "from diffusion_utilities import ResidualConvBlock, UnetUp, UnetDown, EmbedFC; "
            "print(ContextUnet.__module__)" % os.path.join(ROOT, "camels-diffusion-model_amd", "compat"))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "cdm_amd" in r.stdout


def test_library_exports_every_header_symbol():
    import cdm_amd
    from cdm_amd import _lib
    lib = cdm_amd.lib()
    protos = _lib.parse_header()
    out = subprocess.run(["nm", "-D", "--defined-only", lib.path], capture_output=True, text=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    missing = set(protos) - exported
    assert not missing, missing
    assert len(protos) >= 45


def test_cpu_module_fails_loudly():
    """No CPU fallback: the product path refuses to run off the HIP engine."""
    import cdm_amd
    m = cdm_amd.ContextUnet(1, 16, 6, 64)
    with pytest.raises(RuntimeError):
        m(torch.zeros(1, 1, 64, 64), torch.zeros(1))


def test_checkpoint_pth_round_trip(tmp_path, golden_dir):
    """Checkpoint format (saved as train_diffusion_condition.py:254-255, loaded as
    sample_power_spectra.py:187-189): torch.save(state_dict) of this model holds the reference's 156 keys in
    the reference's order, shapes and dtypes, loads with weights_only=True, and a reference-made state_dict
    (golden, produced by the reference's own ContextUnet) loads into this model unchanged."""
    import cdm_amd
    from oracle.ref_cpu import state_dict_layout
    torch.manual_seed(5)
    m = cdm_amd.ContextUnet(1, 16, 6, 64)
    torch.save(m.state_dict(), tmp_path / "model_epoch_99.pth")
    sd = torch.load(tmp_path / "model_epoch_99.pth", weights_only=True)
    layout = state_dict_layout(1, 16, 6, 64)
    assert [k for k, _, _ in layout] == list(sd.keys())
    for k, shape, _ in layout:
        assert tuple(sd[k].shape) == shape, k
        assert sd[k].dtype == (torch.int64 if k.endswith("num_batches_tracked") else torch.float32), k
    fx = np.load(os.path.join(golden_dir, "model_nf16.npz"))
    ref = {k[3:]: torch.from_numpy(fx[k].copy()) for k in fx.files if k.startswith("sd.")}
    m2 = cdm_amd.ContextUnet(1, 16, 6, 64)
    m2.load_state_dict(ref)
    for k, v in m2.state_dict().items():
        assert torch.equal(v, ref[k]), k


def test_cpu_blocks_fail_loudly():
    """The standalone block forwards run on the HIP kernels only (no CPU fallback)."""
    from cdm_amd import EmbedFC, ResidualConvBlock, UnetDown
    for mod, args in ((ResidualConvBlock(4, 8), (torch.zeros(1, 4, 8, 8),)), (UnetDown(4, 8), (torch.zeros(1, 4, 8, 8),)),
                      (EmbedFC(6, 8), (torch.zeros(2, 6),))):
        with pytest.raises(RuntimeError):
            mod(*args)
    blk = ResidualConvBlock(4, 8)
    blk.set_out_channels(16)                      # diffusion_utilities.py:72-75: attributes only
    assert blk.conv1[0].out_channels == blk.conv2[0].in_channels == blk.conv2[0].out_channels == 16


def test_in_channels_layout_and_shortcut_draws():
    """ContextUnet(in_channels > 1): the reference's state_dict layout, the engine's padded image channels (layer specs
    and the NHWC image layout, round-tripped), and the shortcut draws — a fresh Conv2d(C, n_feat, 1) from the CPU RNG
    (the same draws as the reference's), none at all when in_channels == n_feat (identity, diffusion_utilities.py:50-52)."""
    import torch
    import cdm_amd
    from cdm_amd import engine as E
    from oracle import ref_cpu as R
    m = cdm_amd.ContextUnet(3, 16, 6, 16)
    lay = R.state_dict_layout(3, 16, 6, 16)
    sd = m.state_dict()
    assert [k for k, *_ in lay] == list(sd.keys())
    assert all(tuple(sd[k].shape) == tuple(shp) for k, shp, _ in lay)
    L = E.conv_layers(16, 16, 4)
    assert (L[0].cin, L[0].kc, L[1].cin) == (4, 0, 16)
    x = torch.randn(2, 3, 16, 16)
    xe = m._to_engine(x)
    assert xe.shape == (2 * 16 * 16, 4) and torch.equal(xe[:, 3], torch.zeros(512))
    assert torch.equal(m._from_engine(xe, 2), x)
    torch.manual_seed(4)
    w, b = m.draw_shortcut("cpu")
    torch.manual_seed(4)
    rw, rb = R.draw_shortcut(3, 16)
    assert torch.equal(w, rw.reshape(-1)) and torch.equal(b, rb)
    same = cdm_amd.ContextUnet(16, 16, 6, 16)
    state = torch.get_rng_state()
    w, b = same.draw_shortcut("cpu")
    assert torch.equal(torch.get_rng_state(), state)
    assert torch.equal(w, torch.eye(16).reshape(-1)) and not b.any()
    import pytest
    with pytest.raises(NotImplementedError):
        m._engine_and_params()            # training loop / samplers: single-channel only
