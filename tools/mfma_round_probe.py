"""Rounding of the matrix-core accumulation (GPU box): is the fp32 accumulate of the 16-bit MFMAs round-to-nearest?

A GEMM of positive operands, C = A B (M 4096, K 256, N 128), on the engine's GEMM entry points, against fp64:
  * fp16-exact operands through h3 (cdm_gemm_x16 nterm 4): every product is exact in fp32, so the only error is the
    accumulation; round-to-nearest gives errors of both signs (mean / rms ~ 0), truncation gives mean / rms ~ -1
  * bf16-exact operands through the one-term bf16 GEMM (nterm 1): the same question for the bf16 MFMA
  * the same operands through the fp32 MFMA GEMM (cdm_gemm_f32) for comparison
  * general fp32 operands through h3 (the production split)
Prints one JSON line per case: relative L2, mean(err) / rms(err), mean(err) / mean(C).

    python tools/mfma_round_probe.py > gpurun_out/mfma_round.json
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import cdm_amd
    lb = cdm_amd.lib()
    s = torch.cuda.current_stream().cuda_stream
    M, K, N = 4096, 256, 128
    g = torch.Generator().manual_seed(3)
    base_a, base_b = torch.rand(M, K, generator=g), torch.rand(K, N, generator=g)
    out = []

    def run(tag, A, Bm, mode):
        A, Bm = A.contiguous().cuda(), Bm.contiguous().cuda()
        C = torch.empty(M, N, device="cuda")
        if mode == "f32":
            assert lb.cdm_gemm_f32(A.data_ptr(), K, M, K, Bm.data_ptr(), N, N, C.data_ptr(), N, None, 1, 0, 1, None,
                                   s) == 0
        else:
            nterm = 4 if mode == "h3" else 1
            wx = torch.empty((K + 15) // 16 * 3 * N * 16, dtype=torch.bfloat16, device="cuda")
            am = torch.zeros(2, device="cuda")
            if nterm == 4:
                lb.cdm_amax_f32(A.data_ptr(), M, K, K, am.data_ptr(), 0, s)
                lb.cdm_amax_f32(Bm.data_ptr(), K, N, N, am.data_ptr() + 4, 0, s)
                lb.cdm_split_f16x2(Bm.data_ptr(), N, K, N, am.data_ptr() + 4, wx.data_ptr(), s)
                aa, aw = am.data_ptr(), am.data_ptr() + 4
            else:
                lb.cdm_split_bf16x3(Bm.data_ptr(), N, K, N, wx.data_ptr(), s)
                aa = aw = None
            assert lb.cdm_gemm_x16(A.data_ptr(), K, M, K, wx.data_ptr(), aa, aw, N, C.data_ptr(), N, None, 1, None,
                                   nterm, s) == 0
        torch.cuda.synchronize()
        ref = A.double().cpu() @ Bm.double().cpu()
        e = C.double().cpu() - ref
        rec = {"case": tag, "gemm": mode, "rel_l2": (e.norm() / ref.norm()).item(),
               "mean_over_rms": (e.mean() / e.pow(2).mean().sqrt()).item(),
               "mean_over_meanC": (e.mean() / ref.mean()).item(),
               "frac_negative": (e < 0).double().mean().item()}
        out.append(rec)
        print(json.dumps(rec), flush=True)

    a16, b16 = base_a.half().float(), base_b.half().float()
    run("fp16-exact operands (accumulation only)", a16, b16, "h3")
    run("fp16-exact operands (accumulation only)", a16, b16, "f32")
    abf, bbf = base_a.bfloat16().float(), base_b.bfloat16().float()
    run("bf16-exact operands (accumulation only)", abf, bbf, "bf16")
    run("bf16-exact operands (accumulation only)", abf, bbf, "f32")
    run("fp32 operands", base_a, base_b, "h3")
    run("fp32 operands", base_a, base_b, "f32")
    sg = torch.randn(M, K, generator=g).half().float()
    run("fp16-exact operands of both signs", sg, b16, "h3")
    run("fp16-exact operands of both signs", sg, b16, "f32")


if __name__ == "__main__":
    main()
