"""Build libcdm_hip.so in-tree for gfx950 (hipcc; no torch extension machinery, no JIT cache).

    python camels-diffusion-model_amd/build.py [--force]

Objects are rebuilt only when a source or header is newer.  The .so lands in
camels-diffusion-model_amd/lib/ (git-ignored, but shipped to the GPU box by gpurun).
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUTDIR = os.path.join(HERE, "lib")
ROOT = os.path.dirname(HERE)
LIBNAME = os.path.join(OUTDIR, "libcdm_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# -fno-slp-vectorize: no packed-fp32 VALU (v_pk_fma/mul_f32) next to the MFMAs — it issues worse than scalar fp32
# there (MI355X_MICROARCH.md price list); A/B on one box: train step 54.16 -> 53.45 ms (tools/ab_bench.sh)
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-fno-slp-vectorize", "-I", CSRC, "-I",
         os.path.join(ROOT, "include"), "-Wno-unused-result"]


def _newest_dep():
    deps = glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(ROOT, "include", "*.h"))
    deps.append(os.path.abspath(__file__))   # the compile flags
    return max((os.path.getmtime(d) for d in deps), default=0.0)


def build(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(OUTDIR, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    hdr_t = _newest_dep()
    jobs = []
    objs = []
    for s in srcs:
        o = os.path.join(OUTDIR, os.path.basename(s) + ".o")
        objs.append(o)
        if force or not os.path.exists(o) or os.path.getmtime(o) < max(os.path.getmtime(s), hdr_t):
            jobs.append([HIPCC, *FLAGS, "-c", s, "-o", o])

    def run(cmd):
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        if verbose and (r.stderr or r.stdout):
            print(r.stderr or r.stdout, file=sys.stderr)

    if jobs:
        with cf.ThreadPoolExecutor(max_workers=min(8, len(jobs))) as ex:
            list(ex.map(run, jobs))
    if jobs or not os.path.exists(LIBNAME) or os.path.getmtime(LIBNAME) < max(os.path.getmtime(o) for o in objs):
        tmp = LIBNAME + ".tmp"
        run([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", *objs, "-o", tmp])
        os.replace(tmp, LIBNAME)
    return LIBNAME


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
