"""Add the golden host's vector-sqrt tables to schedule.npz (build container; no reference import needed).

    python tests/golden/add_sqrt_tables_r5.py

The reference's denoise_add_noise (code/train_diffusion_condition.py:274-279) takes ``b_t.sqrt()[t]``: torch's
vectorised CPU sqrt of the whole vector, which is not correctly rounded and differs between hosts in a few entries
(round 5, tools/traj_diag.py: the MI355X box's host and this container disagree in sqrt(b_t), sqrt(a_t) and
sqrt(1 - ab_t); the 0-d forms ``a_t[t].sqrt()`` / ``(1 - ab_t[t]).sqrt()`` are IEEE on both).  The golden trajectories
were made here, so the trajectory parity tests replay this container's ``b_t.sqrt()`` (sb_T) — the table the reference
consumed — through diffusion.Schedule(sb=...), exactly as they replay its b_t / a_t / ab_t (add_schedules_r4.py).
``sab_T`` (= ab_t.sqrt(), perturb_input's vector form) is stored for the record.
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import ref_cpu as R  # noqa: E402


def main():
    path = os.path.join(HERE, "schedule.npz")
    fx = dict(np.load(path))
    for T in (10, 400, 1000, 1500, 2000):
        b, a, ab = (torch.from_numpy(fx[f"{k}_{T}"].copy()) for k in ("b_t", "a_t", "ab_t"))
        b2, a2, ab2 = R.make_schedule(T)           # this container reproduces the stored schedule
        assert torch.equal(b, b2) and torch.equal(a, a2) and torch.equal(ab, ab2), T
        fx[f"sb_{T}"] = b.sqrt().numpy()
        fx[f"sab_{T}"] = ab.sqrt().numpy()
        cr = np.sqrt(b.double().numpy()).astype(np.float32)
        print(T, "entries of b_t.sqrt() that are not correctly rounded on this host:", int((cr != fx[f"sb_{T}"]).sum()))
    fx["sqrt_tables_cpu_capability"] = np.array(torch.backends.cpu.get_cpu_capability())
    np.savez(path, **fx)


if __name__ == "__main__":
    main()
