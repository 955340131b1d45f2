"""Debug driver: one nf=128, B=2 h3 train step (fused BN backward) — run with CDM_TRACE_CALLS=1."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from cdm_amd import ContextUnet  # noqa: E402

torch.manual_seed(6)
m = ContextUnet(1, 128, 6, 64, conv_math="h3").cuda().train()
g = torch.Generator().manual_seed(12)
x = torch.rand(2, 1, 64, 64, generator=g).cuda(); c = torch.rand(2, 6, generator=g).cuda()
t = torch.rand(2, generator=g).cuda(); noise = torch.randn(2, 1, 64, 64, generator=g).cuda()
pred = m(x, t, c)
F.mse_loss(pred, noise).backward()
torch.cuda.synchronize()
print("ok", float(m.up0[0].weight.grad.abs().max()))
