"""ctypes binding of libcdm_hip.so.

The argument types are parsed from ``include/cdm_hip.h`` at load time, so the Python side cannot
drift from the C ABI.  Every call checks the returned hipError_t and raises.  There is no CPU
fallback: if the library is missing, :func:`lib` raises, and every op of the package fails loudly.
"""
from __future__ import annotations

import ctypes
import os
import re
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
_ROOT = os.path.dirname(_HERE)
HEADER = os.path.join(_ROOT, "include", "cdm_hip.h")
LIBPATH = os.path.join(_HERE, "lib", "libcdm_hip.so")

_CTYPE = {
    "int": ctypes.c_int, "long long": ctypes.c_longlong, "unsigned long long": ctypes.c_ulonglong,
    "unsigned int": ctypes.c_uint, "float": ctypes.c_float, "double": ctypes.c_double,
}


def parse_header(path: str = HEADER):
    """{name: [ctypes types]} for every ``int cdm_*(...)`` prototype in the header."""
    txt = open(path).read()
    txt = re.sub(r"/\*.*?\*/", " ", txt, flags=re.S)
    protos = {}
    for m in re.finditer(r"\bint\s+(cdm_\w+)\s*\(([^)]*)\)\s*;", txt):
        name, args = m.group(1), m.group(2).strip()
        types = []
        if args and args != "void":
            for a in args.split(","):
                a = " ".join(a.split())
                if "*" in a:
                    types.append(ctypes.c_void_p)
                    continue
                base = re.sub(r"\s+\w+$", "", a).replace("const ", "").strip()
                if base not in _CTYPE:
                    raise ValueError(f"unsupported C type {base!r} in {name}")
                types.append(_CTYPE[base])
        protos[name] = types
    return protos


class HipError(RuntimeError):
    pass


class _Lib:
    def __init__(self, path: str):
        import torch  # noqa: F401  (load torch's HIP runtime first so both share one libamdhip64)
        self._dll = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        self.path = path
        self.protos = parse_header()
        for name, types in self.protos.items():
            fn = getattr(self._dll, name)
            fn.argtypes = types
            fn.restype = ctypes.c_int
            setattr(self, name, self._checked(name, fn))

    @staticmethod
    def _checked(name, fn):
        if os.environ.get("CDM_TRACE_CALLS") == "1":   # debugging: name every call, synchronise after it
            import sys
            import torch

            def traced(*args):
                print("[cdm]", name, args, file=sys.stderr, flush=True)
                rc = fn(*args)
                torch.cuda.synchronize()
                if rc != 0:
                    raise HipError(f"{name} failed with hipError_t {rc}")
                return rc
            traced.__name__ = name
            return traced

        def call(*args):
            rc = fn(*args)
            if rc != 0:
                raise HipError(f"{name} failed with hipError_t {rc}")
            return rc
        call.__name__ = name
        return call

    def raw(self, name):
        return getattr(self._dll, name)


_lock = threading.Lock()
_inst = None


def lib() -> _Lib:
    """The loaded library (raises if it has not been built — there is no fallback path)."""
    global _inst
    if _inst is None:
        with _lock:
            if _inst is None:
                path = os.environ.get("CDM_LIB") or LIBPATH   # A/B timing of two builds (tools); unset in the product
                if not os.path.exists(path):
                    raise RuntimeError(
                        f"libcdm_hip.so not found at {path}; build it with "
                        "`python camels-diffusion-model_amd/build.py` (or __graft_entry__.build())")
                _inst = _Lib(path)
    return _inst


# ------------------------------------------------------------------------------------------------
# EmbedFC descriptor (matches struct MlpDesc / Mlp4 in csrc/misc.hip)
# ------------------------------------------------------------------------------------------------
class MlpDesc(ctypes.Structure):
    _fields_ = [
        ("x", ctypes.c_void_p), ("rows", ctypes.c_int), ("in_dim", ctypes.c_int), ("E", ctypes.c_int),
        ("w1", ctypes.c_void_p), ("b1", ctypes.c_void_p), ("w2", ctypes.c_void_p), ("w2t", ctypes.c_void_p),
        ("b2", ctypes.c_void_p), ("pre", ctypes.c_void_p), ("h", ctypes.c_void_p), ("out", ctypes.c_void_p),
        ("dout", ctypes.c_void_p), ("dpre", ctypes.c_void_p), ("dw1", ctypes.c_void_p), ("db1", ctypes.c_void_p),
        ("dw2", ctypes.c_void_p), ("db2", ctypes.c_void_p),
    ]


class Mlp4(ctypes.Structure):
    _fields_ = [("m", MlpDesc * 4)]
