"""Golden vectors for the sample-statistics row, produced by the REFERENCE itself.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_stats.py        (build container only)

  * ``power_spectrum`` / ``compare_power_spectra`` are imported from the reference's
    ``code/diffusion_utilities.py`` (torchvision stubbed as in make_golden.py);
  * ``calculate_power_spectrum_2d`` is AST-lifted from ``code/sample_power_spectra.py`` and
    ``compare_distributions`` from ``code/train_diffusion.py`` (both scripts run at import time);
  * the plotting calls are served by a recording stand-in for ``plt``, so the arrays the reference
    itself computed and plotted (PDF mean / std per bin, P(k) std bands) are captured as outputs;
    compare_power_spectra also returns its means directly.
Inputs are seeded synthetic maps in [0, 1) (the reference's min-max range; the CAMELS maps are Git-LFS
stubs).  Only inputs and outputs are written (``stats.npz``).
"""
from __future__ import annotations

import os
import sys
import tempfile

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import REF, _lift, _stub_torchvision  # noqa: E402


class _Rec:
    """Records every call made on it (and on anything it returns) — a stand-in for matplotlib."""

    def __init__(self, log, name="plt"):
        self._log, self._name = log, name

    def __getattr__(self, attr):
        def call(*a, **k):
            self._log.append((self._name + "." + attr, a, k))
            if attr == "subplots":
                n = a[1] if len(a) > 1 else 1
                return _Rec(self._log, "fig"), [_Rec(self._log, f"ax{i}") for i in range(n)]
            return _Rec(self._log, self._name + "." + attr)
        return call


def main():
    import numpy as np
    _stub_torchvision()
    sys.path[:0] = [os.path.join(REF, "code"), REF]
    import diffusion_utilities as du  # noqa: E402  (reference)

    rng = np.random.default_rng(2024)
    out = {}

    def maps(n, N):
        """Smooth-ish synthetic maps (a few random Fourier modes + noise), min-max normalised to [0, 1)."""
        xs = np.arange(N)
        res = []
        for _ in range(n):
            m = rng.normal(size=(N, N)) * 0.3
            for _k in range(6):
                kx, ky = rng.integers(1, 8, size=2)
                ph = rng.uniform(0, 2 * np.pi)
                m += np.cos(2 * np.pi * (kx * xs[:, None] + ky * xs[None, :]) / N + ph) * rng.uniform(0.5, 2)
            m = (m - m.min()) / (m.max() - m.min() + 1e-6)
            res.append(m.astype(np.float32))
        return np.stack(res)

    orig, gen = maps(4, 64), maps(4, 64)
    out["orig"], out["gen"] = orig, gen
    box32 = maps(1, 32)[0]
    out["box32"] = box32
    # power_spectrum (diffusion_utilities.py:302-368), dl = 1 and 0.5
    for tag, box, dl in (("ps_a", orig[0], 1.0), ("ps_b", gen[1], 0.5), ("ps_c", box32, 1.0)):
        k, pk = du.power_spectrum(box, dl)
        out[tag + "_k"], out[tag + "_pk"], out[tag + "_dl"] = k, pk, np.float64(dl)
    # compare_power_spectra (diffusion_utilities.py:370-448): returns (k, orig mean, gen mean); the std
    # bands are the fill_between arguments (mean - std, mean + std) over k[1:]
    log = []
    du.plt = _Rec(log)
    with tempfile.TemporaryDirectory() as td:
        import torch
        # documented input: torch tensors [B, 1, H, W] (diffusion_utilities.py:375-376, squeezed at :382-385)
        k, om, gm = du.compare_power_spectra(torch.from_numpy(orig[:, None]), torch.from_numpy(gen[:, None]), td,
                                             dl=1.0)
    out["cps_k"], out["cps_orig_mean"], out["cps_gen_mean"] = k, om, gm
    fb = [c[1] for c in log if c[0] == "plt.fill_between"]
    out["cps_orig_std"] = (np.asarray(fb[0][2]) - np.asarray(fb[0][1])) / 2
    out["cps_gen_std"] = (np.asarray(fb[1][2]) - np.asarray(fb[1][1])) / 2
    # calculate_power_spectrum_2d (sample_power_spectra.py:112-165), lifted
    ns = {"np": np}
    _lift(os.path.join(REF, "code", "sample_power_spectra.py"), ["calculate_power_spectrum_2d"], ns)
    for tag, img, dl in (("p2d_a", orig[2], 1.0), ("p2d_b", gen[3], 0.25)):
        kc, pv = ns["calculate_power_spectrum_2d"](img, dl)
        out[tag + "_k"], out[tag + "_pk"], out[tag + "_dl"] = kc, pv, np.float64(dl)
    # compare_distributions (train_diffusion.py:196-236), lifted; arrays captured from its plot calls
    log = []
    ns = {"np": np, "plt": _Rec(log), "os": os}
    _lift(os.path.join(REF, "code", "train_diffusion.py"), ["compare_distributions"], ns)
    with tempfile.TemporaryDirectory() as td:
        ns["compare_distributions"](orig, gen, td)
    ax0 = [c[1] for c in log if c[0] == "ax0.plot"]
    ax1 = [c[1] for c in log if c[0] == "ax1.plot"]
    out["pdf_bin_mid"] = np.asarray(ax0[0][0])
    out["pdf_train_mean"], out["pdf_test_mean"] = np.asarray(ax0[0][1]), np.asarray(ax0[1][1])
    out["pdf_train_std"], out["pdf_test_std"] = np.asarray(ax1[0][1]), np.asarray(ax1[1][1])
    # round 4: the 3-D branch and non-square boxes of power_spectrum (diffusion_utilities.py:316-363), from a
    # generator of their own (the arrays above are unchanged)
    r3 = np.random.default_rng(2025)
    for tag, shape, dl in (("ps3_a", (16, 20, 24), 0.5), ("ps3_b", (24, 24, 24), 1.0), ("ps_ns", (24, 40), 1.0)):
        box = r3.uniform(0, 1, size=shape).astype(np.float32)
        k, pk = du.power_spectrum(box, dl)
        out[tag + "_box"], out[tag + "_k"], out[tag + "_pk"], out[tag + "_dl"] = box, k, pk, np.float64(dl)
    np.savez_compressed(os.path.join(HERE, "stats.npz"), **out)
    print({k: np.shape(v) for k, v in out.items()})


if __name__ == "__main__":
    main()
