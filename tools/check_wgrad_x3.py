"""Diagnostic: split-bf16 wgrad vs fp32 wgrad over shapes (GPU box)."""
import os, sys, itertools
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cdm_amd
L = cdm_amd.lib(); s = torch.cuda.current_stream().cuda_stream
for N, H, ci, co, spl in itertools.product((1, 2), (8, 16, 32), (32, 128), (64, 128), (1, 7)):
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(N * H * H, ci, device="cuda", generator=g); dy = torch.randn(N * H * H, co, device="cuda", generator=g)
    sp = L.raw("cdm_gemm_splits")(N * H * H, spl)
    s1 = torch.zeros(sp, co, 9 * ci, device="cuda"); s2 = torch.zeros(sp, co, 9 * ci, device="cuda")
    L.cdm_conv3x3_wgrad(dy.data_ptr(), co, co, x.data_ptr(), N, H, H, ci, ci, sp, s1.data_ptr(), s)
    L.cdm_conv3x3_wgrad_x3(dy.data_ptr(), co, co, x.data_ptr(), N, H, H, ci, ci, sp, s2.data_ptr(), 6, s)
    torch.cuda.synchronize()
    a, b = s1.sum(0), s2.sum(0)
    e = (a - b).abs().max().item() / a.abs().max().item()
    bad = (a - b).abs() > 1e-3 * a.abs().max()
    where = bad.nonzero()[:3].tolist() if bad.any() else []
    print(f"N{N} H{H} ci{ci} co{co} sp{sp}: rel {e:.2e} bad {int(bad.sum())} first {where}", flush=True)
