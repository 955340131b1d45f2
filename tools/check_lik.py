"""Diagnostic: per-batch NLL of the GPU evaluator vs the CPU oracle on the golden setup (GPU box)."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import cdm_amd
from oracle import ref_cpu as R
from cdm_amd.likelihood import LikelihoodEvaluator
GOLD = os.path.join(ROOT, "tests", "golden")
fx = np.load(os.path.join(GOLD, "model_nf8.npz"))
sd = {k[3:]: torch.from_numpy(fx[k].copy()) for k in fx.files if k.startswith("sd.")}
lfx = np.load(os.path.join(GOLD, "likelihood_nf8.npz"))
m = cdm_amd.ContextUnet(1, 8, 6, 64); m.load_state_dict(sd); m = m.cuda().eval()
fn = R.make_model_fn(R.clone_sd(sd), n_feat=8, n_cfeat=6, height=64)
T = 10
sched = R.make_schedule(T)
for j in (1, 0):
    x = torch.from_numpy(lfx[f"lik_x{j}"]); c = torch.from_numpy(lfx[f"lik_c{j}"])
    for use_c in (True, False):
        for graph in (True, False):
            ev = LikelihoodEvaluator(m, T, "host", use_graph=graph)
            torch.manual_seed(600 + j)
            got = ev.batch_nll(x, c if use_c else None).cpu()
            torch.manual_seed(600 + j)
            ref = R.calculate_likelihood(fn, [(x, c if use_c else None)], T, sched)
            print(f"batch{j} B={x.shape[0]} c={use_c} graph={graph}: gpu mean {got.mean().item():.6f} oracle {ref:.6f}")
    # single forward at t=T with c
    torch.manual_seed(5)
    with torch.no_grad():
        e1 = m(x.cuda(), torch.tensor([0.5]).cuda(), c.cuda()).cpu()
    torch.manual_seed(5)
    e2 = fn(x, torch.tensor([0.5]), c)
    print(f"batch{j} forward rel {(e1 - e2).abs().max().item() / e2.abs().max().item():.2e}")
