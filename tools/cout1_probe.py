"""out.3's band kernel (C_out = 1 conv) at the bench shape, 16- vs 32-channel slabs ($CDM_COUT1_SLAB, read per call):
mean of 50 back-to-back launches between HIP events, plain and with out.1's GroupNorm + ReLU staged, and the
algorithmic read rate (z read once: N H W C fp32).
    python tools/cout1_probe.py > gpurun_out/cout1.jsonl"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import cdm_amd
    L = cdm_amd.lib()
    s = torch.cuda.current_stream().cuda_stream
    N, H, C = 256, 64, 128
    z = torch.randn(N * H * H, C, device="cuda")
    w = torch.randn(C, 9, device="cuda") * 0.1; b = torch.randn(1, device="cuda")
    gs = torch.rand(N, C, device="cuda") + 0.5; gt = torch.randn(N, C, device="cuda") * 0.1
    out = torch.empty(N, H, H, device="cuda")
    for rnd in range(2):
        for sl in ("16", "32"):
            os.environ["CDM_COUT1_SLAB"] = sl
            for gn in (False, True):
                def go():
                    if gn:
                        return L.cdm_conv3x3_cout1_fwd_gn(z.data_ptr(), C, N, H, H, C, gs.data_ptr(), gt.data_ptr(),
                                                          w.data_ptr(), b.data_ptr(), out.data_ptr(), s)
                    return L.cdm_conv3x3_cout1_fwd(z.data_ptr(), C, N, H, H, C, w.data_ptr(), b.data_ptr(),
                                                   out.data_ptr(), s)
                for _ in range(5):
                    assert go() == 0
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(50):
                    go()
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) / 50 * 1e3
                print(json.dumps({"round": rnd, "slab": int(sl), "gn": gn, "us": round(us, 1),
                                  "TB_s": round(z.numel() * 4 / us / 1e6, 2)}), flush=True)
    del os.environ["CDM_COUT1_SLAB"]


if __name__ == "__main__":
    main()
