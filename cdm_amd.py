"""Import shim: exposes the package directory ``camels-diffusion-model_amd/`` as ``cdm_amd``."""
import importlib.util as _ilu
import os as _os
import sys as _sys

_PKG = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "camels-diffusion-model_amd")
_spec = _ilu.spec_from_file_location("cdm_amd", _os.path.join(_PKG, "__init__.py"), submodule_search_locations=[_PKG])
_mod = _ilu.module_from_spec(_spec)
_sys.modules["cdm_amd"] = _mod
_spec.loader.exec_module(_mod)
