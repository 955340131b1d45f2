"""Bit-exactness of a kernel-row weight-gradient schedule knob at kernel level: runs cdm_conv3x3_wgrad_x16_ex (with
and without the producer BatchNorm sums, PreBnReluSums) on the train step's shapes for h3 and bf16 and writes every
slab / sums buffer to an npz; compare two runs made under two environment settings:
  CDM_WGRAD_STAGGER=0 python tools/wgrad_sched_check.py --out a.npz
  CDM_WGRAD_STAGGER=1 python tools/wgrad_sched_check.py --out b.npz
  python tools/wgrad_sched_check.py --cmp a.npz b.npz"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

ap = argparse.ArgumentParser()
ap.add_argument("--out")
ap.add_argument("--cmp", nargs=2)
a = ap.parse_args()
if a.cmp:
    x, y = np.load(a.cmp[0]), np.load(a.cmp[1])
    bad = [k for k in x.files if not np.array_equal(x[k].view(np.uint32), y[k].view(np.uint32))]
    for k in bad:
        d = np.abs(x[k] - y[k])
        print(f"  {k}: {int((d > 0).sum())} of {d.size} differ, max |d| {d.max():.3e} (max |x| {np.abs(x[k]).max():.3e})")
    print(f"{len(x.files)} buffers, {len(bad)} differ")
    sys.exit(0)
import torch  # noqa: E402

import cdm_amd  # noqa: E402
from cdm_amd.engine import wgrad_splits  # noqa: E402

L = cdm_amd.lib()
st = torch.cuda.current_stream().cuda_stream
out = {}
for nterm in (4, 1):
    for (B, S, cin, cout) in [(16, 64, 128, 128), (16, 32, 256, 256), (16, 32, 128, 256), (16, 16, 256, 256)]:
        g = torch.Generator(device="cuda").manual_seed(5)
        P = B * S * S
        y = torch.randn(P, cin, device="cuda", generator=g)
        gx = torch.randn(P, cin, device="cuda", generator=g)
        dy = torch.randn(P, cout, device="cuda", generator=g) * 1e-2
        s_ = torch.rand(cin, device="cuda", generator=g) + 0.5
        t_ = torch.randn(cin, device="cuda", generator=g) * 0.1
        mean = torch.randn(cin, device="cuda", generator=g) * 0.1
        inv = torch.rand(cin, device="cuda", generator=g) + 0.5
        am = torch.ones(4, device="cuda") * 8.0
        sp = wgrad_splits(P, cout, 9 * cin)
        nt = sp * 3 * (cout // 128)
        for ws in (True, False):
            slab = torch.empty(sp * cout * 9 * cin, device="cuda")
            sums = torch.full((nt * 5 * cin,), float("nan"), device="cuda")
            rc = L.cdm_conv3x3_wgrad_x16_ex(dy.data_ptr(), cout, None, 0, None, None, None, None, None, None, None, cout,
                                            y.data_ptr(), B, S, S, cin, cin, s_.data_ptr(), t_.data_ptr(),
                                            gx.data_ptr() if ws else None, cin, mean.data_ptr() if ws else None,
                                            inv.data_ptr() if ws else None, sums.data_ptr() if ws else None,
                                            am.data_ptr(), am.data_ptr() + 4, sp, slab.data_ptr(), nterm, 0, st)
            assert rc == 0, rc
            torch.cuda.synchronize()
            tag = f"nt{nterm}_B{B}_S{S}_{cin}x{cout}_{'sums' if ws else 'plain'}"
            out[tag + "_slab"] = slab.cpu().numpy()
            if ws:
                out[tag + "_sums"] = sums.cpu().numpy()
np.savez(a.out, **out)
print(f"{len(out)} buffers -> {a.out}")
