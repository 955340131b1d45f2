"""Golden vectors for the data-pipeline row, produced by executing the REFERENCE's own lines.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_data.py        (build container only)

code/train_diffusion_condition.py runs at import time, so the module-level statements of its data section
are compiled straight from the reference file (AST nodes by line number) and executed on synthetic inputs:
  :114-132  parameter expansion / normalisation / column selection     -> param_data_normalized
  :137-144  map shift, /max, log10, min-max, bilinear resize to 64x64   -> camels_data_resized
  :147-156  TensorDataset + random_split(seed 42) of 1500 test maps     -> train / test indices
(the np.save of param_min / param_max goes to a temporary directory).  Writes data.npz.
"""
from __future__ import annotations

import ast
import os
import sys
import tempfile

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import REF  # noqa: E402


def _run_lines(path, lo, hi, ns):
    with open(path) as f:
        tree = ast.parse(f.read(), filename=path)
    body = [n for n in tree.body if lo <= n.lineno <= hi]
    exec(compile(ast.Module(body=body, type_ignores=[]), path, "exec"), ns)
    return ns


def main():
    import numpy as np
    import torch
    import torch.nn.functional as F
    from torch.utils.data import TensorDataset, random_split

    script = os.path.join(REF, "code", "train_diffusion_condition.py")
    rng = np.random.default_rng(7)
    out = {}
    # maps: log-normal-ish positive fields with a few negative / zero pixels (exercise the shift branch)
    raw = (np.exp(rng.normal(size=(6, 256, 256)) * 1.5) * 3e-5).astype(np.float32)
    raw[0, :4, :4] = 0.0
    raw[1, 10, 10] = -1e-6
    raw_pos = (raw[:2] + 2e-6).astype(np.float32)
    raw_pos[raw_pos <= 0] = 1e-7
    params = rng.uniform(0.1, 3.0, size=(2, 6))
    with tempfile.TemporaryDirectory() as td:
        for tag, maps in (("shift", raw), ("pos", raw_pos)):
            ns = {"np": np, "torch": torch, "F": F, "camels_data": maps.copy()}
            _run_lines(script, 137, 144, ns)
            out[f"{tag}_raw"] = maps
            out[f"{tag}_out"] = ns["camels_data_resized"].numpy()
        for num_params in (6, 4):
            ns = {"np": np, "os": os, "param_data": params.copy(), "camels_data": np.zeros((30, 1)),
                  "output_dir": td, "num_params": num_params}
            _run_lines(script, 114, 132, ns)
            out[f"params_norm_{num_params}"] = np.asarray(ns["param_data_normalized"])
            out["param_min"], out["param_max"] = ns["param_min"], ns["param_max"]
        out["params_raw"] = params
    # the split: 1500 of a 3000-map dataset
    n = 3000
    ns = {"torch": torch, "TensorDataset": TensorDataset, "random_split": random_split,
          "camels_data_resized": torch.zeros(n, 1, 1, 1), "param_data_tensor": torch.zeros(n, 1)}
    _run_lines(script, 147, 156, ns)
    out["split_n"] = np.int64(n)
    out["split_train"] = np.asarray(ns["train_dataset"].indices)
    out["split_test"] = np.asarray(ns["test_dataset"].indices)
    np.savez_compressed(os.path.join(HERE, "data.npz"), **out)
    print({k: np.shape(v) for k, v in out.items()})


if __name__ == "__main__":
    main()
