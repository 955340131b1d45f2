"""Run only the ConvT 2x2 forward of up2 at the bench shape (B = 256, 32^2 -> 64^2, 256 -> 128 channels, h3 on the
two-deep prefetch GEMM) N times — the workload of the PMC passes in tools/pmc_convT.sh.
    python tools/convT_only.py [N]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(n=5, B=256, Hin=32, Cin=256, Cout=128):
    import cdm_amd
    L = cdm_amd.lib()
    s = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device="cuda").manual_seed(7)
    M = B * Hin * Hin
    x = torch.randn(M, Cin, device="cuda", generator=g)
    W = torch.randn(Cin, Cout, 2, 2, device="cuda", generator=g) * 0.05
    b = torch.zeros(Cout, device="cuda")
    wt = torch.empty(Cin, 4 * Cout, device="cuda"); wtT = torch.empty(4 * Cout, Cin, device="cuda")
    L.cdm_pack_convT(W.data_ptr(), Cin, Cout, 4, wt.data_ptr(), wtT.data_ptr(), s)
    am = torch.zeros(2, device="cuda")
    L.cdm_amax_f32(wt.data_ptr(), Cin, 4 * Cout, 4 * Cout, am.data_ptr() + 4, 0, s)
    wx = torch.empty((Cin + 15) // 16 * 3 * 4 * Cout * 16, dtype=torch.bfloat16, device="cuda")
    L.cdm_split_f16x2(wt.data_ptr(), 4 * Cout, Cin, 4 * Cout, am.data_ptr() + 4, wx.data_ptr(), s)
    L.cdm_amax_f32(x.data_ptr(), M, Cin, Cin, am.data_ptr(), 0, s)
    y = torch.empty(4 * M, Cout, device="cuda")
    for _ in range(n):
        assert L.cdm_convT2x2_fwd_x16(x.data_ptr(), B, Hin, Hin, Cin, Cin, wx.data_ptr(), am.data_ptr(),
                                      am.data_ptr() + 4, b.data_ptr(), y.data_ptr(), Cout, Cout, None, 4, s) == 0
    torch.cuda.synchronize()


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 5)
