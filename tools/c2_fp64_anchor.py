"""fp64 anchor of the C2 bench-shape gradients (GPU box; a measurement, not a test: the fp64 oracle step at B=256 takes
minutes on the box host's 16 CPUs, beyond what one pytest case may run silently).

The first bench-identical Trainer step (tests/test_gpu_c2_e2e.py::_hip_steps) vs the CPU oracle's full train step in
fp64 and in fp32 from the same weights and draws: per-tensor relative L2 of every parameter gradient for HIP and for the
reference's own fp32 arithmetic, both against fp64.  Writes one JSON object to argv[1] (default
gpurun_out/r3_c2_fp64_anchor.json); prints a heartbeat every 30 s while the oracle runs.

    python tools/c2_fp64_anchor.py [out.json]
"""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import test_gpu_c2_e2e as E  # noqa: E402


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "r3_c2_fp64_anchor.json")
    torch.set_num_threads(16)
    t0 = time.time()
    stop = threading.Event()

    def beat():
        while not stop.wait(30):
            print(f"[anchor {time.time() - t0:6.0f} s] oracle running", flush=True)
    threading.Thread(target=beat, daemon=True).start()
    hip = E._hip_steps()
    st = hip["steps"][0]
    print(f"[anchor {time.time() - t0:6.0f} s] HIP steps done", flush=True)
    l32, p32, g32, _ = E._oracle_step1(torch.float32)
    print(f"[anchor {time.time() - t0:6.0f} s] fp32 oracle done", flush=True)
    l64, p64, g64, _ = E._oracle_step1(torch.float64)
    print(f"[anchor {time.time() - t0:6.0f} s] fp64 oracle done", flush=True)
    stop.set()
    errs, errs32, zero = E._grad_errs(E._grads(hip["tr"], st["gflat"]), g64, g32)
    keys = sorted(errs, key=errs.get)
    res = {"what": "C2 step 1 at B=256, n_feat=128, h3: per-tensor gradient rel L2 vs the fp64 oracle",
           "hip_max": max(errs.values()), "hip_max_tensor": keys[-1], "hip_median": float(np.median(list(errs.values()))),
           "ref32_max": max(errs32.values()), "ref32_max_tensor": max(errs32, key=errs32.get),
           "ref32_median": float(np.median(list(errs32.values()))),
           "hip_over_ref32_median_of_ratios": float(np.median([errs[k] / max(errs32[k], 1e-30) for k in errs])),
           "loss_hip": st["loss"], "loss_fp32": l32, "loss_fp64": l64,
           "per_tensor": {k: {"hip": errs[k], "ref32": errs32[k]} for k in keys}}
    os.makedirs(os.path.dirname(out), exist_ok=True)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "per_tensor"}), flush=True)


if __name__ == "__main__":
    main()
