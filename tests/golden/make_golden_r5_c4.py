"""Round-5 fixture for the C4 (bf16) benchmarked trajectory (build container; CPU only, no reference import).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_r5_c4.py [w]     (w = 0: the default; 3: the CFG golden)

sampler_T1500_nf128_bf16emu.npz — the trajectory of tests/golden/sampler_T1500_nf128.npz (n_feat = 128 seeded default
init, n = 2, w = 0, T = 1500, the golden's schedule, CPU-RNG replay with the golden's seed) re-run by the CPU oracle
under C4's bf16 operand rounding (tests/_bf16emu.py: every 3x3 conv with C_in > 1 and every ConvTranspose2d take bf16
operands, fp32 accumulate): the reference's own sampler at C4's precision, whose deviation from the golden's fp64 re-run
is the bar of tests/test_gpu_configs.py::test_c4_bf16_nf128_T1500_vs_emulated_reference.  Stored: the final x and the
golden's 13 snapshots.  The seeded weights are this package's ContextUnet init, bit-identical to the reference's
(tests/test_api_cpu.py::test_seeded_init_equals_reference).
"""
from __future__ import annotations

import os
import sys
import time

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]


def main(w: float = 0.0):
    import numpy as np
    import torch
    import cdm_amd
    import _parity
    from _bf16emu import _bf16_operands
    from oracle import ref_cpu as R

    torch.set_num_threads(int(os.environ.get("CDM_GOLDEN_THREADS", "8")))
    g = np.load(os.path.join(HERE, "sampler_T1500_nf128.npz" if w == 0 else f"sampler_T1500_nf128_w{w:g}.npz"))
    T, nf = int(g["T"]), int(g["n_feat"])
    torch.manual_seed(int(g["init_seed"]))
    sd = {k: v.detach().clone() for k, v in cdm_amd.ContextUnet(1, nf, 6, 64).state_dict().items()}
    t0 = time.time()
    with _bf16_operands():
        torch.manual_seed(int(g[f"w{w:g}_seed"]))
        x, inter = R.sample_ddpm(R.make_model_fn(R.clone_sd(sd), n_feat=nf, n_cfeat=6, height=64), 2, 64,
                                 torch.from_numpy(g["params"]), w, T, _parity.golden_schedule(T), 6)
    keep = [int(s) for s in g["snap_keep"]]
    k = f"w{w:g}"
    out = {f"{k}_x_bf16emu": x.numpy(), f"{k}_inter_bf16emu": inter.numpy()[keep], "snap_keep": g["snap_keep"],
           "T": g["T"], "n_feat": g["n_feat"]}
    ref = g[f"{k}_x_fp64"]
    print(f"w={w:g}: emulated bf16 run {time.time() - t0:.0f} s; final deviation from fp64 "
          f"{np.abs(out[f'{k}_x_bf16emu'] - ref).max() / np.abs(ref).max():.3e}")
    name = "sampler_T1500_nf128_bf16emu.npz" if w == 0 else f"sampler_T1500_nf128_w{w:g}_bf16emu.npz"
    np.savez_compressed(os.path.join(HERE, name), **out)


if __name__ == "__main__":
    main(float(sys.argv[1]) if len(sys.argv) > 1 else 0.0)
