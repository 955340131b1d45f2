"""Run only the dominant kernel (conv3x3 128->128 @64x64, B=256, train-mode stats epilogue) N times.
Used for PMC passes (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE) that price its HBM traffic per launch."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(n=10, B=256, H=64, C=128, variant=-1, nterm=0):
    import cdm_amd
    L = cdm_amd.lib()
    s = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device="cuda").manual_seed(7)
    x = torch.randn(B * H * H, C, device="cuda", generator=g)
    W = torch.randn(C, C, 3, 3, device="cuda", generator=g) * 0.05
    b = torch.zeros(C, device="cuda")
    wpk = torch.empty(9 * C, C, device="cuda")
    L.cdm_pack_conv3x3(W.data_ptr(), b.data_ptr(), C, C, None, None, None, None, 0.0, wpk.data_ptr(), None, None,
                       16 if variant in (-1, 3, 4) else 0, s)
    y = torch.empty(B * H * H, C, device="cuda")
    st = torch.empty((B * H * H + 127) // 128, 2, C, device="cuda")
    wx = torch.empty(9 * C // 16 * 3 * C * 16, dtype=torch.bfloat16, device="cuda")
    L.cdm_split_bf16x3(wpk.data_ptr(), C, 9 * C, C, wx.data_ptr(), s)
    am = torch.empty(2, device="cuda")
    if nterm == 4:         # h3: scaled fp16 split (amax of x and of the packed weights)
        L.cdm_amax_f32(wpk.data_ptr(), 9 * C, C, C, am.data_ptr() + 4, 0, s)
        L.cdm_split_f16x2(wpk.data_ptr(), C, 9 * C, C, am.data_ptr() + 4, wx.data_ptr(), s)
        L.cdm_amax_f32(x.data_ptr(), B * H * H, C, C, am.data_ptr(), 0, s)
    for _ in range(n):
        if nterm == 4:
            L.cdm_conv3x3_fwd_h3(x.data_ptr(), B, H, H, C, C, wx.data_ptr(), am.data_ptr(), am.data_ptr() + 4,
                                 b.data_ptr(), y.data_ptr(), C, C, 0, st.data_ptr(), C, 16, None, s)
        elif nterm:          # split-bf16 path (conv_math x6 / x3 / bf16)
            L.cdm_conv3x3_fwd_x3(x.data_ptr(), B, H, H, C, C, wx.data_ptr(), b.data_ptr(), y.data_ptr(), C, C, 0,
                                 st.data_ptr(), C, 16, nterm, s)
        elif variant < 0:    # the fp32 path
            L.cdm_conv3x3_fwd(x.data_ptr(), B, H, H, C, C, wpk.data_ptr(), b.data_ptr(), y.data_ptr(), C, C, 0,
                              st.data_ptr(), C, 16, s)
        else:
            L.cdm_conv3x3_fwd_variant(variant, x.data_ptr(), B, H, H, C, C, wpk.data_ptr(), b.data_ptr(),
                                      y.data_ptr(), C, C, 0, st.data_ptr(), C, s)
    torch.cuda.synchronize()
    print("done", n)


if __name__ == "__main__":
    # argv: [n] [variant (fp32 path) | x6 | x3 | x1 | h3]
    arg = sys.argv[2] if len(sys.argv) > 2 else "-1"
    nt = 4 if arg == "h3" else (int(arg[1:]) if arg.startswith("x") else 0)
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 10, variant=-1 if nt else int(arg), nterm=nt)
