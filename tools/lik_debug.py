"""Debug: tests/test_gpu_likelihood.py::test_caller_schedule_is_used under different device-memory contents (an
uninitialised read would make the result depend on what earlier allocations left behind)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import ref_cpu as R  # noqa: E402


def run(tag):
    import cdm_amd
    torch.manual_seed(4)
    m = cdm_amd.ContextUnet(1, 16, 6, 64).cuda().eval()
    sd = R.clone_sd(m.state_dict())
    g = torch.Generator().manual_seed(6)
    batches = [(torch.rand(3, 1, 64, 64, generator=g), torch.rand(3, 6, generator=g))]
    T = 12
    b = (0.03 - 2e-4) * torch.linspace(0, 1, T + 1) + 2e-4
    a = 1 - b
    ab = torch.cumprod(a, 0)
    ab[0] = 1
    fn = R.make_model_fn(sd, n_feat=16, n_cfeat=6, height=64)
    torch.manual_seed(78)
    got = cdm_amd.calculate_likelihood(m, batches, T, "cuda", ab.cuda(), b.cuda(), a.cuda(), noise_source="host")
    torch.manual_seed(78)
    ref = R.calculate_likelihood(fn, batches, T, (b, a, ab))
    torch.manual_seed(78)
    got2 = cdm_amd.calculate_likelihood(m, batches, T, "cuda", ab.cuda(), b.cuda(), a.cuda(), noise_source="host")
    print(f"{tag}: got {got:.6f} again {got2:.6f} ref {ref:.6f} rel {abs(got - ref) / abs(ref):.2e}", flush=True)


run("fresh")
for v in (float("nan"), 1e30, -7.0):
    junk = torch.full((2 ** 31,), v, device="cuda")   # 8 GiB of garbage, then released to the caching allocator
    del junk
    run(f"after fill {v}")
