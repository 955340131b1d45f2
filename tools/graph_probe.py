"""Probe: does a captured cdm_zero_f32 (hipMemsetAsync) node zero its buffer on every replay?  And the sampler's
amax slots after graph runs vs eager."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
import cdm_amd  # noqa: E402
L = cdm_amd.lib()
buf = torch.ones(192, device="cuda")
other = torch.ones(8, device="cuda")
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=s):
    L.cdm_zero_f32(buf.data_ptr(), buf.numel(), torch.cuda.current_stream().cuda_stream)
    other.mul_(2)
torch.cuda.synchronize()
print("after capture (not replayed):", float(buf.sum()), float(other.sum()), flush=True)
g.replay(); torch.cuda.synchronize()
print("after replay 1:", float(buf.sum()), float(other.sum()), flush=True)
buf.fill_(3.0); torch.cuda.synchronize()
g.replay(); torch.cuda.synchronize()
print("after fill 3 + replay 2:", float(buf.sum()), float(other.sum()), flush=True)

fx = np.load("tests/golden/model_nf8.npz")
m = cdm_amd.ContextUnet(1, 8, 6, 64)
m.load_state_dict({k[3:]: torch.from_numpy(fx[k].copy()) for k in fx.files if k.startswith("sd.")})
m = m.cuda().eval()
params = torch.rand(2, 6, generator=torch.Generator().manual_seed(3))
xT = torch.randn(2, 1, 64, 64, generator=torch.Generator().manual_seed(4))
for use_graph in (False, True):
    smp = cdm_amd.GraphSampler(m, cdm_amd.Schedule(20, "cuda"), 2, 0.0, params, z_source="device", seed=7,
                               use_graph=use_graph, steps_per_graph=10)
    for k in range(2):
        torch.manual_seed(5)
        smp.prepare_rng(host_z=False)
        x, inter = smp.run(xT)
        torch.cuda.synchronize()
        n = len(smp.ws.aslot)
        print("graph" if use_graph else "eager", "run", k, "amax slots", np.array2string(smp.ws.amax[:n].cpu().numpy(),
              precision=4, max_line_width=200), flush=True)
