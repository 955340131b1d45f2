"""Probe: is the eval forward / graph sampler bit-deterministic across identical calls?"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import cdm_amd  # noqa: E402

fx = np.load("tests/golden/model_nf8.npz")
m = cdm_amd.ContextUnet(1, 8, 6, 64)
m.load_state_dict({k[3:]: torch.from_numpy(fx[k].copy()) for k in fx.files if k.startswith("sd.")})
m = m.cuda().eval()
x = torch.from_numpy(fx["x"]).cuda(); t = torch.from_numpy(fx["t"]).cuda(); c = torch.from_numpy(fx["c"]).cuda()
outs = []
for k in range(4):
    torch.manual_seed(11)
    with torch.no_grad():
        outs.append(m(x, t, c).clone())
print("eval forward repeat equal:", [torch.equal(outs[0], o) for o in outs[1:]], flush=True)
params = torch.rand(2, 6, generator=torch.Generator().manual_seed(3))
xT = torch.randn(2, 1, 64, 64, generator=torch.Generator().manual_seed(4))
for zs in ("host", "device"):
    d = cdm_amd.DDPM(m, 20, "cuda", z_source=zs)
    res = []
    for k in range(3):
        torch.manual_seed(5)
        o, inter = d.sample_ddpm_from_noise(xT, params, guide_w=0.0)
        res.append((o.cpu(), inter))
        smp = list(d._samplers.values())[0]
        print(zs, "call", k, "zseed", int(smp.zseed), flush=True)
    for k in (1, 2):
        dif = [float(np.abs(res[0][1][j] - res[k][1][j]).max()) for j in range(res[0][1].shape[0])]
        print(zs, f"call0 vs call{k}: per-snapshot max|d|", ["%.1e" % v for v in dif], flush=True)
# eager vs graph within one sampler config
for use_graph in (True, False):
    smp = cdm_amd.GraphSampler(m, cdm_amd.Schedule(20, "cuda"), 2, 0.0, params, z_source="device", seed=7,
                               use_graph=use_graph, steps_per_graph=10)
    r = []
    for k in range(2):
        torch.manual_seed(5)
        smp.prepare_rng(host_z=False)
        r.append(smp.run(xT)[1])
    print("graph" if use_graph else "eager", "repeat max|d| per snapshot",
          ["%.1e" % float(np.abs(r[0][j] - r[1][j]).max()) for j in range(r[0].shape[0])], flush=True)
