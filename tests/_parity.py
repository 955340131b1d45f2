"""Measured parity errors of the GPU tests, recorded for the round's profiles/ (e.g. profiles/r3_parity.json).

Tests call record(name, **values) with the errors they assert on and the bars they hold them to; when $CDM_PARITY_OUT
names a file, each record is appended to it as one JSON line (the GPU run writes it under gpurun_out/, then it is
copied into profiles/).  Without the variable nothing is written."""
import json
import os


def _plain(v):
    try:
        import numpy as np
        if isinstance(v, np.generic):
            return v.item()
    except ImportError:
        pass
    if isinstance(v, dict):
        return {str(k): _plain(x) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return [_plain(x) for x in v]
    return v


def golden_schedule(T: int):
    """(b_t, a_t, ab_t) fp32 CPU tensors the golden trajectories were made with (tests/golden/schedule.npz).

    The schedule is computed on the host with torch's vectorised fp32 log / exp / sqrt, whose last bit depends on the
    host's instruction set (tests/golden/add_schedules_r4.py): a trajectory test compares against a golden made on
    another host only on that host's schedule, passed to the sampler as the reference's functional sampler takes it."""
    import numpy as np
    import torch
    fx = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "schedule.npz"))
    return tuple(torch.from_numpy(fx[f"{k}_{T}"].copy()) for k in ("b_t", "a_t", "ab_t"))


def golden_sqrt_b(T: int):
    """b_t.sqrt() as the golden host's torch evaluated it (tests/golden/add_sqrt_tables_r5.py): the vector-sqrt table
    the reference's denoise_add_noise consumed when the golden trajectories were made (diffusion.Schedule(sb=...))."""
    import numpy as np
    import torch
    fx = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "schedule.npz"))
    return torch.from_numpy(fx[f"sb_{T}"].copy())


def record(name: str, **values):
    path = os.environ.get("CDM_PARITY_OUT")
    if not path:
        return
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "a") as f:
        f.write(json.dumps({"test": name, **_plain(values)}) + "\n")
