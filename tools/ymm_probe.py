"""Cost of the per-column max / min (ymm) epilogue of the h3 LDS-halo conv at the C2 shape (256 x 64^2, 128 -> 128):
the same launch with and without ymm (both with the BN-stats epilogue), HIP events, interleaved rounds."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import cdm_amd  # noqa: E402

L = cdm_amd.lib()
s = torch.cuda.current_stream()
N, H, C = 256, 64, 128
P = N * H * H
g = torch.Generator(device="cuda").manual_seed(3)
x = torch.randn(P, C, device="cuda", generator=g).relu_()
W = torch.randn(9 * C, C, device="cuda", generator=g) * 0.05
am = torch.empty(2, device="cuda")
L.cdm_amax_f32(W.data_ptr(), 9 * C, C, C, am.data_ptr() + 4, 0, s.cuda_stream)
L.cdm_amax_f32(x.data_ptr(), P, C, C, am.data_ptr(), 0, s.cuda_stream)
wx = torch.empty(9 * C // 16 * 3 * C * 16, dtype=torch.bfloat16, device="cuda")
L.cdm_split_f16x2(W.data_ptr(), C, 9 * C, C, am.data_ptr() + 4, wx.data_ptr(), s.cuda_stream)
b = torch.zeros(C, device="cuda")
y = torch.empty(P, C, device="cuda")
stats = torch.empty((P + 127) // 128, 2, C, device="cuda")
ymm = torch.empty(2, C, dtype=torch.int32, device="cuda")
amy = torch.zeros(1, device="cuda")


def launch(with_ymm):
    L.cdm_conv3x3_fwd_h3_ex(x.data_ptr(), N, H, H, C, C, None, None, wx.data_ptr(), am.data_ptr(), am.data_ptr() + 4,
                            b.data_ptr(), y.data_ptr(), C, C, 0, stats.data_ptr(), C, 16, amy.data_ptr(),
                            ymm.data_ptr() if with_ymm else None, C, s.cuda_stream)


for w in (False, True):
    for _ in range(3):
        launch(w)
res = {False: [], True: []}
for r in range(5):
    for w in (False, True):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(20):
            launch(w)
        e1.record(s)
        e1.synchronize()
        res[w].append(e0.elapsed_time(e1) / 20)
for w in (False, True):
    v = sorted(res[w])
    print(f"ymm={w}: median {v[len(v) // 2]:.4f} ms  all {[round(t, 4) for t in res[w]]}", flush=True)
