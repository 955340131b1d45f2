"""Reference-named shim for code/diffusion_utilities.py: the hot-path building blocks (lines 13-145).

The analysis helpers of that file (plotting, power spectra, datasets; lines 147-448) are outside the
accelerated path and are not provided here."""
import os as _os
import sys as _sys

_ROOT = _os.path.dirname(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))))
if _ROOT not in _sys.path:
    _sys.path.insert(0, _ROOT)
import cdm_amd as _cdm  # noqa: E402

ResidualConvBlock = _cdm.ResidualConvBlock
UnetUp = _cdm.UnetUp
UnetDown = _cdm.UnetDown
EmbedFC = _cdm.EmbedFC
__all__ = ["ResidualConvBlock", "UnetUp", "UnetDown", "EmbedFC"]
