"""Reference-named shim: `from ContextUnet import ContextUnet` (ContextUnet.py:5) -> the HIP engine model.

Put this directory on sys.path; the repository root must be importable too."""
import os as _os
import sys as _sys

_ROOT = _os.path.dirname(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))))
if _ROOT not in _sys.path:
    _sys.path.insert(0, _ROOT)
import cdm_amd as _cdm  # noqa: E402

ContextUnet = _cdm.ContextUnet
__all__ = ["ContextUnet"]
