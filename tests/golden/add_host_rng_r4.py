"""Host CPU-RNG draws of the sampler goldens' order (build container; no reference import needed).

    python tests/golden/add_host_rng_r4.py

torch's CPU normal sampler (torch.randn, Box-Muller with vectorised log / sin / cos) is last-bit dependent on the host's
instruction set, like the schedule (add_schedules_r4.py).  host_rng.npz keeps the first draws of the T = 1500 golden's
run (seed 700: x_T, the step-1500 z, the step's shortcut) as made on the container that made the goldens, so a GPU-box
test can count how many of its own draws differ (tests/test_gpu_sampler.py::test_host_rng_vs_golden).
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import ref_cpu as R  # noqa: E402


def draws():
    torch.manual_seed(700)
    x_T = torch.randn(2, 1, 64, 64)
    z = torch.randn(2, 1, 64, 64)
    w, b = R.draw_shortcut(1, 8)
    return {"x_T": x_T.numpy(), "z_1500": z.numpy(), "sc_w": w.numpy(), "sc_b": b.numpy(),
            "small": torch.randn(8).numpy()}


def main():
    fx = draws()
    fx["cpu_capability"] = np.array(torch.backends.cpu.get_cpu_capability())
    np.savez(os.path.join(HERE, "host_rng.npz"), **fx)
    print({k: v.shape for k, v in fx.items()})


if __name__ == "__main__":
    main()
