"""CAMELS data pipeline on the device, code/train_diffusion_condition.py:104-160.

    preprocess_maps(maps, size=64) -> cuda [N, 1, size, size] fp32
        lines 137-144: shift to positive, / max, log10, min-max to [0, 1], bilinear resize — one min/max
        reduction over the raw maps + one fused normalise-and-interpolate pass (csrc/data.hip)
    preprocess_params(params, n_maps, num_params, out_dir=None) -> [N, num_params] fp32
        lines 112-134: repeat x15, per-column min-max (param_min.npy / param_max.npy saved), select / pad columns
    train_test_split(n, test_size=1500, seed=42) -> (train_idx, test_idx)
        line 152-156: torch.utils.data.random_split with a seeded generator (the same permutation)
    params_txt_to_npy(txt, npy) -> array
        code/txt-npy.py:1-11: whitespace-separated parameter table -> .npy

The maps are processed in the dtype the reference sees for a float32 .npy (fp32).  The raw maps are uploaded
once (3.9 GB for the full 15000 x 256^2 set, of 288 GB HBM); the min / max reduction is over the whole dataset,
as in the reference, and the normalise-and-resize pass runs in chunks of `chunk` maps.
"""
from __future__ import annotations

import os
from typing import Tuple

import numpy as np
import torch

from ._lib import lib


def _s():
    return torch.cuda.current_stream().cuda_stream


def preprocess_maps(maps, size: int = 64, chunk: int = 2048) -> torch.Tensor:
    """Device restatement of code/train_diffusion_condition.py:137-144 for maps [N, S, S]."""
    if torch.is_tensor(maps):
        x = maps.detach().to("cuda", torch.float32).contiguous()
    else:
        x = torch.from_numpy(np.ascontiguousarray(np.asarray(maps, dtype=np.float32))).cuda()
    if x.dim() == 4:
        x = x[:, 0]
    N, S = x.shape[0], x.shape[-1]
    if x.dim() != 3 or x.shape[1] != S:
        raise ValueError("expected maps [N, S, S]")
    keys = torch.empty(2, dtype=torch.int32, device=x.device)
    mm = torch.empty(2, device=x.device)
    lb = lib()
    lb.cdm_minmax_f32(x.data_ptr(), x.numel(), keys.data_ptr(), mm.data_ptr(), _s())
    out = torch.empty(N, 1, size, size, device=x.device)
    for i in range(0, N, chunk):
        n = min(chunk, N - i)
        lb.cdm_camels_maps(x[i:i + n].data_ptr(), n, S, size, mm.data_ptr(), out[i:i + n].data_ptr(), _s())
    return out


def preprocess_params(params: np.ndarray, n_maps: int, num_params: int, out_dir: str = None) -> torch.Tensor:
    """code/train_diffusion_condition.py:112-134 (host: a [N/15, 6] table)."""
    expanded = np.repeat(params, 15, axis=0)
    assert expanded.shape[0] == n_maps, "Parameter expansion doesn't match image count"
    pmin = expanded.min(axis=0, keepdims=True)
    pmax = expanded.max(axis=0, keepdims=True)
    norm = (expanded - pmin) / (pmax - pmin + 1e-8)
    if out_dir:
        np.save(os.path.join(out_dir, "param_min.npy"), pmin)
        np.save(os.path.join(out_dir, "param_max.npy"), pmax)
    if norm.shape[1] > num_params:
        norm = norm[:, :num_params]
    elif norm.shape[1] < num_params:
        norm = np.concatenate([norm, np.zeros((norm.shape[0], num_params - norm.shape[1]))], axis=1)
    return torch.tensor(norm, dtype=torch.float32)


def train_test_split(n: int, test_size: int = 1500, seed: int = 42) -> Tuple[torch.Tensor, torch.Tensor]:
    """The index sets of random_split(full, [n - test, test], generator=manual_seed(seed)) (:150-156)."""
    perm = torch.randperm(n, generator=torch.Generator().manual_seed(seed))
    return perm[: n - test_size], perm[n - test_size:]


def params_txt_to_npy(txt_path: str, npy_path: str) -> np.ndarray:
    """code/txt-npy.py:1-11 — np.loadtxt of the whitespace-separated table (float64), saved as .npy."""
    data = np.loadtxt(txt_path)
    np.save(npy_path, data)
    return data
