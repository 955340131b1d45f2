"""Probe: does a hipGraph capture / replay move torch's CUDA generator so that manual_seed + random_ differs?"""
import torch
t = torch.zeros(1, dtype=torch.int64, device="cuda")
torch.manual_seed(5); t.random_(); a = int(t)
x = torch.zeros(4, device="cuda")
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.graph(g, stream=s):
    x.add_(1)
g.replay(); g.replay()
torch.manual_seed(5); t.random_(); b = int(t)
torch.manual_seed(5); t.random_(); c = int(t)
print("random_ after seed: before capture", a, "after capture", b, "again", c, flush=True)
import sys
sys.path.insert(0, ".")
import numpy as np, cdm_amd
m = cdm_amd.ContextUnet(1, 8, 6, 64).cuda().eval()
d = cdm_amd.DDPM(m, 20, "cuda")
params = torch.rand(2, 6); xT = torch.randn(2, 1, 64, 64)
for k in range(3):
    torch.manual_seed(5)
    out, _ = d.sample_ddpm_from_noise(xT, params, guide_w=0.0)
    smp = list(d._samplers.values())[0]
    print("call", k, "zseed", int(smp.zseed), "sum", float(out.double().sum()), flush=True)
