"""Round-5 golden vectors from the REFERENCE itself (build container only; needs /root/reference): the CFG companion of
make_golden_r5.py (same model, schedule and method; guide weight w = 3, seed 901).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_r5_w3.py

sampler_T1500_nf128_w3.npz — the benchmarked CFG trajectory: sample_ddpm (code/train_diffusion_condition.py:281-335,
AST-lifted as in make_golden.py) of the reference ContextUnet at n_feat = 128 (seeded default init,
torch.manual_seed(0); the HIP model's seeded init is the same, tests/test_api_cpu.py), n = 2, guide weight w = 3 (cond + uncond halves of one batched forward),
T = 1500 steps of the reference schedule, CPU-RNG order of the reference's CPU run.  Stored: params, the x_T seed, the
final x and 13 of the 82 snapshots, plus the same trajectory re-run by the CPU oracle in fp64 (oracle/ref_cpu.py fed
the same draws), whose distance to the fp32 reference is the reference's own fp32 accuracy — the tolerance basis of
tests/test_gpu_sampler.py::test_sample_nf128_T1500_matches_reference.  The weights are not stored (67 MB): the test
rebuilds them from the seed.  The schedule and its b_t.sqrt() table are this container's (tests/golden/schedule.npz).

Nothing from the reference is written to the repo except these numeric outputs.
"""
from __future__ import annotations

import os
import sys
import time

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from make_golden import REF, _lift, _stub_torchvision  # noqa: E402

NF, NCF, T = 128, 6, 1500
SNAP_KEEP = (0, 1, 5, 25, 50, 74, 75, 76, 77, 78, 79, 80, 81)   # of the 82 snapshots at T = 1500, save_rate = 20


def main():
    _stub_torchvision()
    sys.path[:0] = [os.path.join(REF, "code"), REF]
    import numpy as np
    import torch
    from ContextUnet import ContextUnet  # noqa: E402  (reference)
    from oracle import ref_cpu as R

    torch.set_num_threads(int(os.environ.get("CDM_GOLDEN_THREADS", "8")))
    torch.manual_seed(0)
    model = ContextUnet(1, NF, NCF, 64)
    model.eval()
    b_t, a_t, ab_t = R.make_schedule(T)
    sch = np.load(os.path.join(HERE, "schedule.npz"))
    assert np.array_equal(ab_t.numpy(), sch[f"ab_t_{T}"]) and np.array_equal(b_t.sqrt().numpy(), sch[f"sb_{T}"])
    cond_script = os.path.join(REF, "code", "train_diffusion_condition.py")
    ns = {"torch": torch, "np": np, "nn_model": model, "b_t": b_t, "a_t": a_t, "ab_t": ab_t, "timesteps": T,
          "n_cfeat": NCF, "device": torch.device("cpu")}
    _lift(cond_script, ["denoise_add_noise", "sample_ddpm"], ns)
    params = torch.rand(2, NCF, generator=torch.Generator().manual_seed(5050))
    sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in model.state_dict().items()}
    sched64 = tuple(v.double() for v in (b_t, a_t, ab_t))
    fx = {"params": params.numpy(), "T": np.array(T), "n_feat": np.array(NF), "init_seed": np.array(0),
          "snap_keep": np.array(SNAP_KEEP)}
    w, seed = 3.0, 901
    t0 = time.time()
    torch.manual_seed(seed)
    xs, inter = ns["sample_ddpm"](n_sample=2, size=64, device=torch.device("cpu"), params=params, guide_w=w)
    assert inter.shape[0] == 82, inter.shape
    fx["w3_seed"] = np.array(seed)
    fx["w3_x"] = xs.numpy()
    fx["w3_inter"] = inter[list(SNAP_KEEP)]
    t1 = time.time()
    print(f"fp32 reference run {t1 - t0:.0f} s", flush=True)
    torch.manual_seed(seed)
    x64 = torch.randn(2, 1, 64, 64).double()

    def model64(xx, t, cc):
        wgt, bias = R.draw_shortcut(1, NF)
        with torch.no_grad():
            return R.unet_forward(sd64, xx, t.double(), cc, n_feat=NF, n_cfeat=NCF, height=64, train=False,
                                  shortcut=(wgt.double(), bias.double()))

    x64f, inter64 = R.sample_loop(model64, x64, params.double(), w, T, sched64, 20,
                                  noise_fn=lambda i, xx: torch.randn(xx.shape).double())
    fx["w3_x_fp64"] = x64f.numpy()
    fx["w3_inter_fp64"] = inter64.numpy()[list(SNAP_KEEP)]
    mx = np.abs(fx["w3_x_fp64"]).max()
    d = np.abs(fx["w3_x"] - fx["w3_x_fp64"]).max() / mx
    print(f"nf=128 T={T} w=3: fp32 {t1 - t0:.0f} s, fp64 {time.time() - t1:.0f} s, max|x| {mx:.4g}, "
          f"fp32 ref vs fp64 max|d|/max|x| {d:.3e}", flush=True)
    np.savez_compressed(os.path.join(HERE, "sampler_T1500_nf128_w3.npz"), **fx)
    print("done")


if __name__ == "__main__":
    main()
