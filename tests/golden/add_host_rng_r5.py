"""SHA-256 of the whole CPU-RNG draw sequence of the T = 1500 trajectory goldens (build container; no reference import).

    python tests/golden/add_host_rng_r5.py

host_rng.npz (add_host_rng_r4.py) keeps the first draws of one seed; this adds, per T = 1500 golden trajectory, one hash
over every draw the reference's CPU run consumes in its order (x_T, then per step the z of steps T..2 and the shortcut
(w, b) of every forward; w = 0: one forward per step), so tests/test_gpu_sampler.py::test_host_rng_vs_golden checks
the complete sequence on the GPU box's host, not only its start.
"""
import hashlib
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import ref_cpu as R  # noqa: E402

# (fixture key, seed, n_feat, T): sampler_T1500_nf8.npz (w = 0), sampler_T1500_nf128.npz and sampler_T1500_nf128_w3.npz
# (CFG: one forward of the 2n batch per step, so the same draw order — x_T, then per step z and one shortcut)
SEQUENCES = (("seq_T1500_nf8_w0", 700, 8, 1500), ("seq_T1500_nf128_w0", 900, 128, 1500),
             ("seq_T1500_nf128_w3", 901, 128, 1500))


def sequence_hash(seed: int, nf: int, T: int, n: int = 2) -> str:
    h = hashlib.sha256()
    torch.manual_seed(seed)
    h.update(torch.randn(n, 1, 64, 64).numpy().tobytes())
    for i in range(T, 0, -1):
        if i > 1:
            h.update(torch.randn(n, 1, 64, 64).numpy().tobytes())
        w, b = R.draw_shortcut(1, nf)
        h.update(w.numpy().tobytes()); h.update(b.numpy().tobytes())
    return h.hexdigest()


def main():
    path = os.path.join(HERE, "host_rng.npz")
    fx = dict(np.load(path))
    for key, seed, nf, T in SEQUENCES:
        fx[key] = np.array(sequence_hash(seed, nf, T))
        print(key, str(fx[key]))
    np.savez(path, **fx)


if __name__ == "__main__":
    main()
