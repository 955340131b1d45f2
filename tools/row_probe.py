"""Standalone timing of the C_in = 1 forward and C_out = 1 input-gradient kernels at the C2 shape (bs 256, 64x64, 128
channels), whichever form $CDM_ROW_KERNELS selects:  python tools/row_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cdm_amd  # noqa: E402

L = cdm_amd.lib()
s = torch.cuda.current_stream().cuda_stream
N, H, C = 256, 64, 128
P = N * H * H
x = torch.randn(P, device="cuda")
w9 = torch.randn(9 * C, device="cuda")
b = torch.randn(C, device="cuda")
y = torch.empty(P, C, device="cuda")
am = torch.zeros(1, device="cuda")
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


def t(fn, reps=10):
    best = 1e9
    for _ in range(reps):
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3)
    return best


f1 = t(lambda: L.cdm_conv3x3_cin1_fwd(x.data_ptr(), N, H, H, w9.data_ptr(), b.data_ptr(), y.data_ptr(), C, C, 1,
                                      am.data_ptr(), s))
f0 = t(lambda: L.cdm_conv3x3_cin1_fwd(x.data_ptr(), N, H, H, w9.data_ptr(), b.data_ptr(), y.data_ptr(), C, C, 1, None, s))
d = t(lambda: L.cdm_conv3x3_cout1_dgrad(x.data_ptr(), N, H, H, C, w9.data_ptr(), y.data_ptr(), C, s))
from cdm_amd.engine import CHUNK  # noqa: E402
nch = -(-H * H // CHUNK)
slab = torch.empty(N * nch * 2 * C, device="cuda")
ymm = torch.zeros(2 * C, dtype=torch.int32, device="cuda")
sm = t(lambda: L.cdm_reduce_stats_mm(y.data_ptr(), C, N, H * H, C, CHUNK, slab.data_ptr(), ymm.data_ptr(), C, s))
nb = P * C * 4
print(f"CDM_ROW_KERNELS={os.environ.get('CDM_ROW_KERNELS', '1')}: cin1_fwd (amax) {f1:.1f} us {nb / f1 / 1e6:.2f} TB/s, "
      f"cin1_fwd {f0:.1f} us, cout1_dgrad {d:.1f} us {nb / d / 1e6:.2f} TB/s, stats_mm {sm:.1f} us {nb / sm / 1e6:.2f} TB/s")
