"""ConvT 2x2 forward (up2 at the bench shape, h3) timed between HIP events, alternating an environment switch read per
call (default CDM_CONVT_DEEP: gemm_x3 vs the two-deep prefetch GEMM): mean of 30 launches per setting, 3 rounds.
Round 5 also used it for non-temporal output stores (a since-removed CDM_CONVT_NT switch): 393.9 / 355.9 / 340.8 us
plain vs 393.4 / 345.2 / 340.3 us non-temporal — no change, the clock ramp across rounds dominates
(profiles/r5_convT_nt_probe.jsonl).
    python tools/convT_probe.py [ENV_NAME]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(env="CDM_CONVT_DEEP", B=256, Hin=32, Cin=256, Cout=128):
    import cdm_amd
    L = cdm_amd.lib()
    s = torch.cuda.current_stream().cuda_stream
    M = B * Hin * Hin
    x = torch.randn(M, Cin, device="cuda")
    W = torch.randn(Cin, Cout, 2, 2, device="cuda") * 0.05
    b = torch.zeros(Cout, device="cuda")
    wt = torch.empty(Cin, 4 * Cout, device="cuda"); wtT = torch.empty(4 * Cout, Cin, device="cuda")
    L.cdm_pack_convT(W.data_ptr(), Cin, Cout, 4, wt.data_ptr(), wtT.data_ptr(), s)
    am = torch.zeros(2, device="cuda")
    L.cdm_amax_f32(wt.data_ptr(), Cin, 4 * Cout, 4 * Cout, am.data_ptr() + 4, 0, s)
    wx = torch.empty((Cin + 15) // 16 * 3 * 4 * Cout * 16, dtype=torch.bfloat16, device="cuda")
    L.cdm_split_f16x2(wt.data_ptr(), 4 * Cout, Cin, 4 * Cout, am.data_ptr() + 4, wx.data_ptr(), s)
    L.cdm_amax_f32(x.data_ptr(), M, Cin, Cin, am.data_ptr(), 0, s)
    y = torch.empty(4 * M, Cout, device="cuda")
    ref = None
    for rnd in range(3):
        for v in ("0", "1"):
            os.environ[env] = v
            go = lambda: L.cdm_convT2x2_fwd_x16(x.data_ptr(), B, Hin, Hin, Cin, Cin, wx.data_ptr(), am.data_ptr(),  # noqa
                                                am.data_ptr() + 4, b.data_ptr(), y.data_ptr(), Cout, Cout, None, 4, s)
            for _ in range(3):
                assert go() == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(30):
                go()
            e1.record()
            torch.cuda.synchronize()
            if ref is None:
                ref = y.clone()
            same = bool(torch.equal(y, ref))
            print(json.dumps({"round": rnd, env: v, "us": round(e0.elapsed_time(e1) / 30 * 1e3, 1), "same": same}),
                  flush=True)
    del os.environ[env]


if __name__ == "__main__":
    main(*sys.argv[1:2])
