"""Scan input seeds of tests/test_gpu_trainer.py::trainer_three_steps for one where no fp32-class arithmetic flips a
ReLU / MaxPool kink (step gradients within a small multiple of the reference's own fp32 deviation) — GPU box.

    python tools/trainer_seed_scan.py [seeds...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_gpu_trainer as T  # noqa: E402

seeds = [int(a) for a in sys.argv[1:]] or list(range(1, 9))
for sd in seeds:
    worst = 0.0
    for math in ("h3", "x6", "fp32"):
        res = T.trainer_three_steps(math, sd)
        for r in res:
            q = max(r["grad_max"] / (r["grad_max_ref32"] + 1e-5), r["grad_median"] / (r["grad_median_ref32"] + 1e-5),
                    r["dev_rms"] / (r["dev_rms_ref32"] + 1e-3), r["dev_p99"] / (r["dev_p99_ref32"] + 1e-3),
                    r["loss_err"] / (r["loss_err_ref32"] + 1e-6 * abs(r["loss64"]) / 3),
                    r["bn_err"] / (r["bn_err_ref32"] + 1e-6 / 3))
            worst = max(worst, q)
            print(f"seed {sd} [{math}] step {r['step']}: grad max {r['grad_max']:.2e} (ref {r['grad_max_ref32']:.2e}) "
                  f"rms {r['dev_rms']:.2e} (ref {r['dev_rms_ref32']:.2e}) p99 {r['dev_p99']:.2e} "
                  f"(ref {r['dev_p99_ref32']:.2e}) loss {r['loss_err']:.2e} (ref {r['loss_err_ref32']:.2e}) BN "
                  f"{r['bn_err']:.2e} (ref {r['bn_err_ref32']:.2e})", flush=True)
    print(f"seed {sd}: worst ratio {worst:.2f} (the test needs <= 3)", flush=True)
