"""CPU oracle (TEST INFRASTRUCTURE ONLY) for the data-pipeline row, SURVEY §8f #2.

Restates code/train_diffusion_condition.py:137-144 (map preprocessing) in the reference's own numpy / torch
operations and dtype; pinned bit-exactly to vectors produced by executing those reference lines
(tests/golden/make_golden_data.py -> data.npz; tests/test_oracle_data.py).  The shipped device pipeline is
cdm_amd.data (csrc/data.hip); this module only checks it.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F


def preprocess_maps(camels_data: np.ndarray, size: int = 64) -> torch.Tensor:
    """code/train_diffusion_condition.py:137-144 (float32 maps stay float32, as in the reference)."""
    x = np.array(camels_data)
    mn = np.min(x)                                          # :137
    if mn <= 0:
        x = x - mn + 1e-8                                   # :139
    x = x / np.max(x)                                       # :140
    x = np.log10(x)                                         # :141
    x = (x - x.min()) / (x.max() - x.min())                 # :142
    t = torch.tensor(x, dtype=torch.float32).unsqueeze(1)   # :143
    return F.interpolate(t, size=(size, size), mode="bilinear")   # :144
